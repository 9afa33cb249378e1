import sys, gc, weakref
sys.path.insert(0, '.')
import torch
from bayesianoptimizer_amd import GPEngine, _capi
from bayesianoptimizer_amd.engine import _FactorBuffer
e = GPEngine(0)
owner = _FactorBuffer(e, (256, 256), _capi.GPX_ALLOC_UNCACHED)
w = weakref.ref(owner)
t = torch.as_tensor(owner, device=e.device)
del owner
gc.collect()
print("owner alive while tensor lives:", w() is not None, "refcount-type", type(t))
v = t[:10, :10]
del t
gc.collect()
print("owner alive with only a view:", w() is not None)
del v
gc.collect()
print("owner alive after all views gone:", w() is not None)
