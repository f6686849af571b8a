"""CPU-only checks: the C-ABI library builds/loads and exports every symbol
include/umamd.h declares; the Python binding covers exactly that set; the
drop-in modules construct with the reference schema; graph loading."""
import os
import re
import subprocess

import pytest

from conftest import PKG, REPO


def _header_symbols():
    src = open(os.path.join(REPO, 'include', 'umamd.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(um_\w+)\s*\(', src)))


def test_library_exports_header_symbols():
    from umamd import _build, _lib
    lib_path = _build.build()
    out = subprocess.run(['nm', '-D', '--defined-only', lib_path], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r'\bT (um_\w+)', out))
    declared = _header_symbols()
    assert declared, 'no declarations parsed'
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    assert sorted(_lib.exported_symbols()) == declared
    L = _lib.lib()  # binds every declared entry (argtypes) without a GPU
    assert L.um_version() == 1


def test_host_queries_without_gpu():
    from umamd._lib import query
    assert query('um_conv_stats_parts', 1000, 32) == 8
    # bf16 stage-1 7x7 conv (halo kernel) and an f32 one (implicit GEMM)
    assert query('um_conv_wgrad_splits', 1, 8, 128, 256, 32, 32, 32, 7, 1, 3, 0, 128, 256, 32) >= 1
    assert query('um_conv_wgrad_splits', 0, 8, 128, 256, 32, 32, 32, 7, 1, 3, 0, 128, 256, 32) >= 1
    assert query('um_conv_fwd_ws', 1, 8, 8, 16, 512, 3, 512) > 0  # deep layer: split-K
    assert query('um_conv_fwd_ws', 1, 8, 128, 256, 32, 7, 32) == 0
    assert query('um_adam_chunk') == 4096
    from umamd.packer import PackDesc
    import ctypes
    assert query('um_pack_desc_size') == ctypes.sizeof(PackDesc)
    assert query('um_colred_ws', 1000, 32, 2) > 0


def test_kernel_call_fails_loudly_on_cpu_tensor():
    import torch
    from umamd import functional as U
    from umamd._lib import UmamdError
    with pytest.raises(UmamdError):
        U.image_to_nhwc(torch.zeros(1, 3, 32, 32), torch.float32)


def test_model_schema_and_param_count():
    import yaml
    import model as M
    from oracle import model as OM, step as OS
    cfg = yaml.safe_load(open(os.path.join(REPO, 'config.yml')))
    cfg['model']['encoder']['load_graph'] = os.path.join(REPO, 'graphs/nodes_5_seed_42')
    m = M.RandomlyConnectedModel(**cfg['model'])
    specs = OS.param_specs(cfg['model'], OM.load_stage_graphs(cfg['model']['encoder']))
    sd = m.state_dict()
    assert list(sd.keys()) == [s[0] for s in specs]
    assert all(tuple(sd[k].shape) == tuple(s[1]) for k, s in zip(sd, specs))
    assert sum(p.numel() for p in m.parameters()) == 22_493_949
    m.load_state_dict(OS.formula_state_dict(specs))
    assert M.Model is M.RandomlyConnectedModel


def test_nodes10_schema():
    import yaml
    import model as M
    from oracle import model as OM, step as OS
    cfg = yaml.safe_load(open(os.path.join(REPO, 'config_nodes10.yml')))
    cfg['model']['encoder']['load_graph'] = os.path.join(REPO, 'graphs/nodes_10_seed_42')
    m = M.RandomlyConnectedModel(**cfg['model'])
    specs = OS.param_specs(cfg['model'], OM.load_stage_graphs(cfg['model']['encoder']))
    assert list(m.state_dict().keys()) == [s[0] for s in specs]
    assert sum(p.numel() for p in m.parameters()) == 35_442_189


@pytest.mark.skipif(not os.path.isdir('/root/reference/graphs'), reason='reference absent')
def test_gpickle_reader_matches_json():
    from model.graph import load_graph
    for s in range(1, 6):
        a = load_graph(f'/root/reference/graphs/nodes_5_seed_42/stage_{s}.gpickle')
        b = load_graph(os.path.join(REPO, f'graphs/nodes_5_seed_42/stage_{s}.json'))
        assert a == b


def test_graph_info_f3_order():
    from model.graph import get_graph_info, load_graph
    from model.layers.encoder import NodeBlock
    g = load_graph(os.path.join(REPO, 'graphs/nodes_5_seed_42/stage_1.json'))
    nodes, ins, outs = get_graph_info(g)
    assert ins == [0] and outs == [4]
    assert [n.inputs for n in nodes] == [[], [0], [1, 0], [2, 1, 0], [3, 0, 2, 1]]
    assert NodeBlock.weight_index(4) == [0, 0, 1, 2]


def test_graph_build_nodes10_matches_committed():
    pytest.importorskip('networkx')
    from model.graph import build_graph, load_graph
    for s in range(1, 6):
        assert build_graph(10, 4, 0.75, 42 * s) == \
            load_graph(os.path.join(REPO, f'graphs/nodes_10_seed_42/stage_{s}.json'))


def test_loss_config_surface():
    import yaml
    from train.loss import TukraUncertaintyLoss
    cfg = yaml.safe_load(open(os.path.join(REPO, 'config.yml')))
    lf = TukraUncertaintyLoss(**cfg['loss'])
    assert lf.predictive_error.loss_type == 'l1'
    assert lf.wssim.previous_image_error is None
    with pytest.raises(ValueError):
        TukraUncertaintyLoss(error_loss_config={'loss_type': 'bogus'})


def test_schedules_match_oracle():
    import train.utils as u
    from oracle import loss as OL
    for e in range(60):
        assert float(u.adjust_disparity(e)) == pytest.approx(OL.adjust_disparity(e))


def test_build_stamp_is_path_independent(tmp_path):
    """The library stamp hashes sources, headers and the flags with the
    include directories relative to the repository: a copy of the tree at
    another path (the GPU box's snapshot) computes the same digest, so it
    loads the shipped libumamd.so instead of rebuilding it."""
    import glob
    import importlib.util
    import shutil
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = os.path.join(repo, 'uncertainty-model_amd')
    dst = tmp_path / 'elsewhere' / 'repo'
    (dst / 'uncertainty-model_amd' / 'csrc').mkdir(parents=True)
    (dst / 'uncertainty-model_amd' / 'umamd').mkdir(parents=True)
    shutil.copytree(os.path.join(repo, 'include'), dst / 'include')
    for f in glob.glob(os.path.join(pkg, 'csrc', '*')):
        if os.path.isfile(f):
            shutil.copy(f, dst / 'uncertainty-model_amd' / 'csrc')
    shutil.copy(os.path.join(pkg, 'umamd', '_build.py'), dst / 'uncertainty-model_amd' / 'umamd')

    def digest(path):
        spec = importlib.util.spec_from_file_location(f'_b{abs(hash(path))}', path)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        return m._digest()
    here = digest(os.path.join(pkg, 'umamd', '_build.py'))
    there = digest(str(dst / 'uncertainty-model_amd' / 'umamd' / '_build.py'))
    assert here == there
