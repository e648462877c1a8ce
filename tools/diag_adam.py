import sys, torch, numpy as np
sys.path.insert(0, '.')
from tests.test_gpu_aggregation import _mixed_model, _noncontig, _msgs_dev
from oracle import aggregation_ref as agg_ref
from fl_sim_amd import aggregation
for n_msgs in (3, 20):
    params = _mixed_model(4)
    g = torch.Generator().manual_seed(5)
    msgs = [{"train_samples": 10, "delta_parameters": [(torch.randn(p.shape, generator=g) * 1e-3).to(p.dtype) for p in params]} for _ in range(n_msgs)]
    dls = [(torch.randn(p.shape, generator=g) * 1e-4).to(p.dtype) for p in params]
    vs = [(torch.rand(p.shape, generator=g) * 1e-4 + 1e-6).to(p.dtype) for p in params]
    betas = (0.9, 0.99)
    exp_p, exp_d, exp_v = [p.clone() for p in params], [d.clone() for d in dls], [v.clone() for v in vs]
    agg_ref.fedopt_update(exp_p, exp_d, exp_v, msgs, "adam", 0.5, betas, 1e-3)
    got_p, got_d, got_v = _noncontig(params), _noncontig(dls), _noncontig(vs)
    aggregation.fedopt_update(got_p, got_d, got_v, _msgs_dev(msgs, "delta_parameters"), "adam", 0.5, betas, 1e-3)
    for name, G, E in (("p", got_p, exp_p), ("d", got_d, exp_d), ("v", got_v, exp_v)):
        for j, (x, y) in enumerate(zip(G, E)):
            a = x.cpu().contiguous().numpy().ravel(); b = y.contiguous().numpy().ravel()
            bad = np.nonzero(a.view(np.uint64 if a.dtype == np.float64 else np.uint32) != b.view(np.uint64 if b.dtype == np.float64 else np.uint32))[0]
            print(n_msgs, name, j, a.dtype, len(bad), bad[:5], a[bad[:3]], b[bad[:3]])
