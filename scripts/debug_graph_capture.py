"""Bisects a crash at HIP-graph capture end in the HCCF plugin's graph mode: the unit-test step
(tests/test_gpu_graph_step.py) with the plugin's differences switched on one at a time.

    python scripts/debug_graph_capture.py {dropout,clip,plugin}
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests import test_gpu_graph_step as T  # noqa: E402
from hypergraph_diffusion_for_recommendation_amd.graphs import CapturedStep  # noqa: E402

dev = torch.device("cuda:0")
what = sys.argv[1]
if what.startswith("plugin"):
    import random
    import tempfile

    from tests import test_gpu_plugins as TP
    from hypergraph_diffusion_for_recommendation_amd.plugins import HCCF
    from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise
    from hypergraph_diffusion_for_recommendation_amd.selfrec import (FileIO, ModelConf,
                                                                     default_args)
    td = tempfile.mkdtemp()
    d = TP._write_dataset(os.path.join(td, "dataset")) + "/"
    with open(os.path.join(td, "HCCF.conf"), "w") as f:
        f.write(TP.HCCF_CONF.format(model="HCCF"))
    conf = ModelConf(os.path.join(td, "HCCF.conf"))
    kw = default_args(dataset='toy', max_epoch=1, batch_size=256, embedding_size=32,
                      hyper_dim=32, n_layers=2, item_ranking='10,20', drop_rate=0.3, p=0.5,
                      temp=0.2, cl_rate=1e-3, reg=0.01, seed=7)
    kw['hgd_graph'] = True
    os.chdir(td)
    rec = HCCF(conf, FileIO.load_data_set(d + "train.txt"), FileIO.load_data_set(d + "test.txt"),
               None, **kw)
    random.seed(3)
    bs = list(next_batch_pairwise(rec.data, 256, device=dev))
    print("batch dtypes", [t.dtype for t in bs[0]], [t.shape for t in bs[0]],
          [t.is_contiguous() for t in bs[0]], flush=True)
    if what == "plugin_selfrec":
        from hypergraph_diffusion_for_recommendation_amd.selfrec import SELFRec
        kw2 = default_args(dataset='toy', max_epoch=2, batch_size=256, embedding_size=32,
                           hyper_dim=32, input_dim=32, n_layers=2, item_ranking='10,20',
                           drop_rate=0.3, p=0.5, temp=0.2, cl_rate=1e-3, reg=0.01,
                           early_stopping_steps=5, seed=7)
        kw2['hgd_graph'] = True
        kw2['dataset_root'] = os.path.join(td, "dataset")
        conf.config['dataset'] = 'toy'
        random.seed(3)
        torch.manual_seed(3)
        import faulthandler
        faulthandler.enable()
        import hypergraph_diffusion_for_recommendation_amd.plugins as PL
        orig = PL.HCCF.graph_step

        def traced(self, u, i, j):
            print("graph_step", getattr(self, "_eager_steps", 0), self._captured is not None,
                  u.shape, u.dtype, u.device, u.is_contiguous(), flush=True)
            return orig(self, u, i, j)
        PL.HCCF.graph_step = traced
        SELFRec(conf, kw2).execute()
        sys.exit(0)
    if what == "plugin_eager":
        rec._eager_steps = -100
    for k, b in enumerate(bs[:5]):
        print(k, float(rec.graph_step(*b)), flush=True)
    sys.exit(0)
enc, U, I = T._hccf(dev, drop_rate=0.3 if what in ("dropout", "clip") else 0.0)
lr = torch.tensor(1e-3, device=dev)
opt = torch.optim.Adam(enc.parameters(), lr=lr, capturable=True)
inner = T._step_fn(enc, opt, U)


def step(u, i, j):
    if what == "clip":
        enc.train()
        torch.nn.utils.clip_grad_norm_(enc.parameters(), 4)
    return inner(u, i, j)


g = torch.Generator(device=dev).manual_seed(7)
batches = [tuple(torch.randint(0, n, (256,), device=dev, generator=g) for n in (U, I, I))
           for _ in range(4)]
print("eager", float(step(*batches[0])), flush=True)
cap = CapturedStep(step, batches[1])
print("captured", [float(cap(*b)) for b in batches[1:]], flush=True)
