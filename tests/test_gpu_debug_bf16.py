"""bf16 vs fp32 HIP path, node by node (localisation aid).  Marked gpu."""
import os

import numpy as np
import pytest
import torch
import yaml

from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max())


def test_bf16_vs_fp32_nodewise():
    import model as M
    from oracle import model as OM, step as OS
    from umamd import functional as U
    with open(os.path.join(REPO, 'config.yml')) as f:
        cfg = yaml.safe_load(f)
    cfg['model']['encoder']['load_graph'] = os.path.join(REPO, cfg['model']['encoder']['load_graph'])
    specs = OS.param_specs(cfg['model'], OM.load_stage_graphs(cfg['model']['encoder']))
    sd = OS.formula_state_dict(specs)
    z = np.load(os.path.join(GOLDEN, 'model_fwd.npz'))
    left = torch.from_numpy(z['left']).cuda()
    res = {}
    for dt in ('fp32', 'bf16'):
        m = M.RandomlyConnectedModel(**cfg['model'], dtype=dt)
        m.load_state_dict(sd)
        m = m.cuda().train()
        with torch.no_grad():
            x = U.image_to_nhwc(left, m.compute_dtype)
            gb = m.encoder.layers[0].layers[0]
            r = {'x': x}
            r[0] = gb.node_blocks[0]._fwd(x)
            for node in gb.nodes[1:]:
                r[node.id] = gb.node_blocks[node.id]._fwd(*[r[i] for i in node.inputs])
            # single conv with the fp32 input
            res[dt] = r
    out = []
    for k in res['fp32']:
        out.append(f'{k}: {_rel(res["bf16"][k], res["fp32"][k]):.3e}')
    # conv of fp32-converted input in bf16 vs fp32
    print('NODES ' + ' | '.join(out))
