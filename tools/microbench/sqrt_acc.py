import ctypes, os, numpy as np, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "sqrt_acc.so"))
t = np.concatenate([np.random.RandomState(0).uniform(0, 80, 2_000_000), 10.0 ** np.random.RandomState(1).uniform(-20, 2, 1_000_000), [0.0]])
dt = torch.from_numpy(t).cuda(); out = torch.zeros(2 * len(t), dtype=torch.float64, device="cuda")
lib.run(ctypes.c_void_p(dt.data_ptr()), ctypes.c_void_p(out.data_ptr()), len(t))
o = out.cpu().numpy().reshape(-1, 2); ref = np.sqrt(t)
nz = ref > 0
print("rsq-newton max ulp", np.max(np.abs(o[nz, 0] - ref[nz]) / np.spacing(ref[nz])), "ocml", np.max(np.abs(o[nz, 1] - ref[nz]) / np.spacing(ref[nz])), "zero ok", o[-1, 0] == 0)
