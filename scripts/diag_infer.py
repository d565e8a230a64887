import sys, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from test_gpu_inference import calibrate, images, oracle_params_from, rel_err, ON
from tf_depth_estimation_amd import batch_prediction as bp, _api, variables, nets_depth
variables.get_store().reset(seed=1); _api.clear_programs()
N, H, W = 1, 96, 128
x = images(N, H, W, 6, 8)
pf = bp.Predictor("depthflow_net", H, W, batch=N, graph=False)
calibrate(pf.prog.chunk, images(8, H, W, 6, 9), 9, lambda P, x: ON.disp_net_depthflow(P, x, True, scope="model/depth_net", decay=0.0))
pf.refresh()
fo = [o.clone() for o in pf(x.cuda())]
with variables.variable_scope("model"):
    un = [o.clone() for o in nets_depth.disp_net(x.cuda(), is_training=False)[0]]
P = oracle_params_from(pf.prog.chunk, "")
ref = ON.disp_net_depthflow(P, x.double(), False, scope="model/depth_net")
for i in range(8):
    r = ref[i]
    sat = ((r < 0.0011) | (r > 10.0)).double().mean().item() if i < 4 else 0
    print(i, "fold-vs-ref %.2e unf-vs-ref %.2e fold-vs-unf %.2e sat %.2f refmax %.3e" % (rel_err(fo[i], r), rel_err(un[i], r), rel_err(fo[i], un[i].double()), sat, r.abs().max().item()))
# per-layer: compare activations of each buffer folded vs unfolded
