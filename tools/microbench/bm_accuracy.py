import ctypes, os, numpy as np, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "bm_accuracy.so"))
rng = np.random.RandomState(0)
u = np.concatenate([rng.uniform(size=2_000_000), 10.0 ** rng.uniform(-16, 0, size=1_000_000),
                    np.array([0.5 * 2 ** -53, 0.125, 0.25, 0.375, 0.5, 0.625, 0.75, 0.875, 1 - 2 ** -53])])
du = torch.from_numpy(u).cuda(); out = torch.zeros(6 * len(u), dtype=torch.float64, device="cuda")
lib.run(ctypes.c_void_p(du.data_ptr()), ctypes.c_void_p(out.data_ptr()), len(u))
o = out.cpu().numpy().reshape(-1, 6)
ref_log = np.log(u); ref_s = np.sin(2 * np.pi * u); ref_c = np.cos(2 * np.pi * u)
def ulp_err(a, b): return np.max(np.abs(a - b) / np.spacing(np.maximum(np.abs(b), 1e-300)))
print("log  custom vs numpy max ulp", ulp_err(o[:, 0], ref_log), " ocml", ulp_err(o[:, 1], ref_log))
print("sin  custom vs ocml max abs", np.max(np.abs(o[:, 2] - o[:, 3])), " vs numpy", np.max(np.abs(o[:, 2] - ref_s)))
print("cos  custom vs ocml max abs", np.max(np.abs(o[:, 4] - o[:, 5])), " vs numpy", np.max(np.abs(o[:, 4] - ref_c)))
