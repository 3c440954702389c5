import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "."); sys.path.insert(0, "i-emic_amd")
from test_gpu_coupled import setup, atmos_oracle
from oracle import atmos_oracle as ao
from iemic.coupled import Atmosphere
c, g, L, oc = setup("coupled4")
atm = Atmosphere(oc, {**ao.COUPLED_RUN_PARAMS, "Combined Forcing": c.start_params["Combined Forcing"]})
at = atmos_oracle(c, g, L)
xa = g["xa"]; rng = np.random.default_rng(5); sst = 0.3 * rng.standard_normal(c.n * c.m)
atm.setState(xa); atm.setOceanTemperature(sst)
F = atm.computeRHS(); oF = at.rhs(xa, sst)
bad = np.nonzero(F != oF)[0]
print("nbad", len(bad))
for r in bad[:40]:
    cell = r // 3; i, j = cell % c.n, cell // c.n
    print(r, r % 3, i, j, at.surf[j, i] if j < c.m else -1, F[r], oF[r], F[r] - oF[r])
