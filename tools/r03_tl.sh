set -o pipefail
mkdir -p gpurun_out
GIBBS_HIP_LIB=gibbssampler_amd/libgibbs_hip_timeline.so timeout -k 10 200 python -u tools/mh_timeline.py > gpurun_out/r03_tl.log 2>&1 || { tail -20 gpurun_out/r03_tl.log; exit 1; }
cat gpurun_out/r03_tl.log
