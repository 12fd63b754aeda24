import ctypes, os, numpy as np, torch, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import harmonic as H
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "xor3_check.so"))
out = torch.zeros(256, dtype=torch.int64, device="cuda").view(torch.int32)
lib.run(ctypes.c_void_p(out.data_ptr()))
got = out.cpu().numpy().view(np.uint32)[:256].reshape(64, 4)
ref = np.stack(H.philox4x32_10(np.arange(64), 0, 0, 0, 0, 0), axis=1).astype(np.uint32)
print("xor3 philox matches oracle:", np.array_equal(got, ref))
