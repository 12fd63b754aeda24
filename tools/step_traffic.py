"""One masked bench step between two marker launches, for HBM-traffic PMC
passes of the WHOLE step (every kernel of it, ring stages and f2 included):

  rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- \\
      python3 tools/step_traffic.py --workload masked_asis --nchains 16 [--mask galactic]
  (then the same with WRITE_SIZE; python tools/summarize_step_traffic.py folds both)

The workload is bench.py's own (masked_head_setup / masked_c5_setup: the same
data, samplers and warm-up); the markers are two k_remove_md launches on a
scratch array (a kernel no masked step runs), so the step's dispatches are the
ones strictly between them.  Arguments: bench.py's (--workload, --nchains,
--nside, --lmax, --mask); one warm-up iteration, one measured step."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import torch
    import bench
    from gibbssampler_amd import _capi
    from gibbssampler_amd.distributed import ShardContext
    sys.argv = ["bench.py", "--no-cpu-baseline", "--steps", "1", "--warmup", "1"] + sys.argv[1:]
    args = bench.parse()
    torch.cuda.set_device(0)
    ctx = ShardContext(args.nchains, backend="nccl")
    lib = _capi.load()
    scratch = torch.zeros(16, dtype=torch.float64, device="cuda")

    def marker():
        _capi.check(lib.gs_remove_monopole_dipole(2, 1, _capi.ptr(scratch), _capi.stream_ptr()), "marker")

    try:
        if args.workload == "masked":
            step = bench.masked_c5_setup(args, ctx)
            step()                                  # warm-up iteration
            torch.cuda.synchronize()
            marker()
            step()
            marker()
            n_sht, ncomp = 2.0, 3
        else:
            runner, go, n_sht, what, pcg = bench.masked_head_setup(args, ctx)
            n0 = len(pcg.pcg_iterations) if pcg is not None else 0
            torch.cuda.synchronize()
            marker()
            go()
            marker()
            ncomp = 2
            if pcg is not None:     # bench.py's count: 2 per CG iteration + 7 for the right-hand side
                import numpy as np
                n_sht = 2 * float(np.mean(pcg.pcg_iterations[n0:])) + 7
        torch.cuda.synchronize()
        import json
        print("STEP_TRAFFIC " + json.dumps({"workload": args.workload, "nside": args.nside, "lmax": args.lmax,
                                           "nchains": args.nchains, "mask": args.mask, "n_sht": n_sht,
                                           "ncomp": ncomp}), flush=True)
    finally:
        ctx.close()


if __name__ == "__main__":
    main()
