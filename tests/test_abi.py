"""C-ABI boundary checks (no GPU needed): include/drpo_hip.h is the single source
of truth; every function it declares must be exported by libdrpo_hip.so and bound
with a ctypes prototype in drpo_amd._abi, and nothing else may be exported."""
import ctypes
import os
import re
import subprocess

import pytest

import drpo_amd
from drpo_amd import _abi, _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'drpo_hip.h')


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', ' ', src, flags=re.S)
    src = re.sub(r'//[^\n]*', ' ', src)
    return sorted(set(re.findall(r'\b(drpo_[a-z0-9_]+)\s*\(', src)))


def exported_symbols():
    out = subprocess.run(['nm', '-D', '--defined-only', _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    return sorted({ln.split()[-1] for ln in out.splitlines() if ln.split() and ln.split()[-1].startswith('drpo_')})


@pytest.fixture(scope='module')
def built():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip('libdrpo_hip.so not built (run __graft_entry__.build())')
    return _lib.lib()


def test_header_matches_exports(built):
    hdr = header_functions()
    assert len(hdr) >= 25
    assert hdr == exported_symbols()


def test_header_matches_ctypes_prototypes(built):
    assert header_functions() == sorted(_abi.PROTOTYPES)
    for name in _abi.PROTOTYPES:
        assert isinstance(getattr(built, name), ctypes._CFuncPtr)


def test_host_only_entry_points(built):
    # these run without a device: version, error string, size queries
    assert built.drpo_version() >= 1
    assert isinstance(built.drpo_last_error(), bytes)
    # the loaded binary was built from exactly the sources in the tree
    from drpo_amd import build_lib
    assert built.drpo_build_digest().decode() == build_lib.source_digest()
    assert built.drpo_grad_sumsq_blocks(2048 * 3 + 1) == 4
    assert built.drpo_normalizer_workspace_size(4096, 12) == 8 * 2 * 12 * 2


def test_header_compiles_as_c():
    """The header is plain C (no HIP/torch types) so cgo/JNI/ctypes users can bind it."""
    r = subprocess.run(['gcc', '-x', 'c', '-std=c99', '-fsyntax-only', '-Wall', '-Werror', '-'],
                       input='#include "drpo_hip.h"\nint main(void){return drpo_version();}\n', text=True,
                       capture_output=True, cwd=os.path.join(ROOT, 'include'), env=dict(os.environ, CPATH=os.path.join(ROOT, 'include')))
    assert r.returncode == 0, r.stderr


def test_device_entry_points_refuse_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    with pytest.raises(_lib.DrpoError):
        _lib.require_device(torch.zeros(1))


def test_struct_layouts_match(built):
    """Every ctypes mirror has the C struct's size (catches field drift in either)."""
    from drpo_amd import _abi as A
    pairs = {'drpo_rollout_desc_t': A.RolloutDesc, 'drpo_mlp_layer_t': A.MlpLayer, 'drpo_mlp_net_t': A.MlpNet,
             'drpo_policy_head_t': A.PolicyHead, 'drpo_mlp_fwd_t': A.MlpFwd, 'drpo_mlp_bwd_layer_t': A.MlpBwdLayer,
             'drpo_mlp_bwd_net_t': A.MlpBwdNet, 'drpo_mlp_bwd_t': A.MlpBwd, 'drpo_wgrad_item_t': A.WgradItem,
             'drpo_buffer_view_t': A.BufferView, 'drpo_critic_head_t': A.CriticHead,
             'drpo_pack_item_t': A.PackItem, 'drpo_pack_map_t': A.PackMap, 'drpo_optim_seg_t': A.OptimSeg,
             'drpo_ens_reduce_t': A.EnsReduce}
    for name, cls in pairs.items():
        assert built.drpo_abi_sizeof(name.encode()) == ctypes.sizeof(cls), name
    assert built.drpo_abi_sizeof(b'nope') == -1


def test_stale_library_is_refused(built, monkeypatch):
    """_lib.lib() loads nothing whose compiled-in source digest differs from the tree's."""
    from drpo_amd import build_lib
    monkeypatch.setattr(build_lib, 'source_digest', lambda: '0' * 64)
    monkeypatch.setattr(_lib, '_lib', None)
    with pytest.raises(_lib.DrpoError, match='built from other sources'):
        _lib.lib()
