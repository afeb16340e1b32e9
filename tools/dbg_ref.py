import sys, os
sys.path[:0]=['.','tests','tests/golden']
import torch, numpy as np
from helpers import golden_weights, rel_err, grad_checks
from test_gpu_training import _load, _model, _x
z=_load("refmode_spring_s12"); dev=torch.device("cuda:0")
for mode in ["reference", "fresh_recons_only"]:
    m=_model(z,dev); m.build_optimizer(1e-3,"rmsprop",True)
    with torch.no_grad():
        m.output=m.conv_feedforward(_x(z["input_u8_eval"],dev))
    stale=m.output
    out=m.forward(_x(z["input_u8_0"],dev))
    if mode=="reference":
        m.loss_mode="reference"; tl,_=m.compute_loss()
    else:
        m.output=out; tl,(p,e,r)=m.compute_loss(); tl = 3.0*r
    m.optimizer.zero_grad(set_to_none=True); tl.backward(); torch.cuda.synchronize()
    grads={k:q.grad for k,q in m.named_parameters() if q.grad is not None}
    print(mode, sorted(grads)==sorted(str(k) for k in z["grad_keys"]))
    errs=grad_checks(z,{k:v for k,v in grads.items() if k in set(str(x) for x in z["grad_keys"])},1e9)
    print(sorted(errs.items(), key=lambda kv:-kv[1])[:8])
