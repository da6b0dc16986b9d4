import numpy as np, sys
sys.path.insert(0,'.')
import torch
from tests.test_gpu_kernels import _run_gpu, _oracle, _ragged
from krr_amd import _native
ctx = _native.Context(0)
rng = np.random.default_rng(5)
offs = _ragged(rng, 200, 0, 3000)
N = int(offs[-1])
vals = rng.integers(0, 3, size=N).astype(np.float64)
special = rng.random(N)
vals[special < 0.02] = -0.0
vals[(special >= 0.02) & (special < 0.025)] = np.inf
vals[(special >= 0.025) & (special < 0.03)] = -np.inf
for mode in ["sorted_lower", "linear"]:
    gv, gn, gf = _run_gpu(ctx, vals, offs, mode, 99, 1)
    wv, wn, wf = _oracle(vals, offs, mode, 99, 1)
    bad = np.nonzero(gf != wf)[0]
    for s in bad[:6]:
        seg = vals[offs[s]:offs[s+1]]
        print(mode, s, "len", len(seg), "flags", hex(gf[s]), "got", gv[s], "want", wv[s], "ninf", np.sum(np.isposinf(seg)), "n2", np.sum(seg==2))
