"""GPU vs oracle bitwise diagnostic for the mixing Jacobian/residual (development tool)."""
import sys, numpy as np
sys.path[:0]=['/root/repo','/root/repo/i-emic_amd','/root/repo/tests']
from iemic import config as cf
from iemic.ocean import Ocean
from oracle import oracle as orc
for name in ["natl8","global4"]:
    c=cf.preset(name); L=cf.init_landmask(c, cf.landmask(c)); x=cf.synthetic_state(c, cf.landmask(c))
    oc=Ocean(c, landm=L, analyze_jacobian=False); o=orc.Oracle(c.ref_dict(), L, c.par_list())
    oc.setState(x); F=oc.computeRHS(); oc.computeJacobian(); _,_,val=oc.exportCSR(); ov,_=o.jacobian(x); oF=o.rhs(x)
    print(name, "J entries differing:", int(np.count_nonzero(val!=ov)), "of", len(ov), "F entries differing:", int(np.count_nonzero(F!=oF)), flush=True)
