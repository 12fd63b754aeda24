import numpy as np, torch, os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from tests.test_gpu_const_rings import _cr, _spec
for mk in ("band", "galactic"):
    cr, mm, dl, s0 = _cr(16, 32, mk, gibbs_cr=False, ula=False, sht_mode="mfma", rng="native")
    print(mk, "classes", cr.ring_classes, "tables", cr.sht_tables)
    dlu = np.stack([dl[k] for k in _spec(2)])
    x = torch.from_numpy(np.ascontiguousarray(s0[1:] * 10)).cuda()
    d = torch.from_numpy(dlu).cuda()
    a = cr.pcg_apply(d, x).cpu().numpy()
    os.environ["GS_SHT_CONST_RINGS"] = "0"
    b = cr.pcg_apply(d, x).cpu().numpy()
    del os.environ["GS_SHT_CONST_RINGS"]
    print(mk, "max diff", np.abs(a - b).max(), np.abs(a).max())
