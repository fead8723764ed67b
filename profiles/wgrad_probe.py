"""Micro-benchmark of drpo_mlp_wgrad (csrc/wgrad.hip) on the SAC critic update's item
set at B rows (config 2: B = 4096) and on single items, timed with HIP events over
back-to-back launches. With DRPO_LIB_OVERRIDE=<...>/libdrpo_hip_stamps.so it also
prints the per-workgroup phase cycles (s_memtime stamps).

python profiles/wgrad_probe.py [rows]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import drpo_amd  # noqa: E402,F401
from drpo_amd import _lib  # noqa: E402
from drpo_amd._abi import WgradItem  # noqa: E402

DEV = torch.device('cuda')
SA = 14      # quadrotor S + A (the input layers' width, not a multiple of 4)
C = 2
# the critic update's items: twin Q nets, constraint-critic trunk, mean / log-std heads
CRITIC = [(256, SA), (256, 256), (1, 256)] * 2 + [(256, SA), (256, 256)] + [(256, 256), (C, 256)] * 2
ACTOR = [(256, 12), (256, 256), (4, 256)] * 2          # actor + safe actor (S = 12, 2A = 4)
MULT = [(256, 13), (256, 256), (1, 256)]               # MLPMultiplier (S + 1 inputs)


def make(shapes, rows):
    out = []
    for dout, din in shapes:
        out.append(dict(dz=torch.randn(rows, dout, device=DEV), y=torch.randn(rows, din, device=DEV),
                        gW=torch.zeros(dout, din, device=DEV), gb=torch.zeros(dout, device=DEV), dout=dout, din=din))
    return out


def items_arr(items, rows):
    arr = (WgradItem * len(items))()
    for k, d in enumerate(items):
        it = arr[k]
        it.dz, it.y, it.gW, it.gb = d['dz'].data_ptr(), d['y'].data_ptr(), d['gW'].data_ptr(), d['gb'].data_ptr()
        it.dout, it.din, it.rows, it.nbatch = d['dout'], d['din'], rows, 1
        it.zstride, it.ystride, it.gwstride, it.gbstride = rows * d['dout'], rows * d['din'], d['dout'] * d['din'], \
            d['dout']
    return arr


def time_launch(items, rows, reps=200):
    L = _lib.lib()
    arr = items_arr(items, rows)
    need = L.drpo_mlp_wgrad_workspace_size(arr, len(items))
    ws = torch.zeros(max(need, 256), dtype=torch.uint8, device=DEV)
    st = _lib.stream()
    for _ in range(10):
        _lib.check(L.drpo_mlp_wgrad(arr, len(items), ws.data_ptr(), ws.numel(), st), 'wgrad')
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        _lib.check(L.drpo_mlp_wgrad(arr, len(items), ws.data_ptr(), ws.numel(), st), 'wgrad')
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    flop = sum(2.0 * rows * d['dout'] * d['din'] for d in items)
    return us, flop / (us * 1e-6) / 1e12


def stamps(items, rows):
    L = _lib.lib()
    if not hasattr(L, 'drpo_debug_stamps_wgrad'):
        return None
    L.drpo_debug_stamps_wgrad.argtypes = [ctypes.c_void_p, ctypes.c_int]
    arr = items_arr(items, rows)
    need = L.drpo_mlp_wgrad_workspace_size(arr, len(items))
    ws = torch.zeros(max(need, 256), dtype=torch.uint8, device=DEV)
    n = 1 << 14
    buf = np.zeros((n, 8), np.uint64)
    L.drpo_debug_stamps_wgrad_clear()
    torch.cuda.synchronize()
    _lib.check(L.drpo_mlp_wgrad(arr, len(items), ws.data_ptr(), ws.numel(), _lib.stream()), 'wgrad')
    torch.cuda.synchronize()
    L.drpo_debug_stamps_wgrad(buf.ctypes.data, n)
    st = buf.astype(np.int64)
    nwg = int((st[:, 0] > 0).sum())
    st = st[:nwg]
    # s_memtime is per XCD (not synchronised across XCDs): per-workgroup differences only
    out = {'workgroups': nwg}

    def stat(a, b, name):
        ok = (st[:, a] > 0) & (st[:, b] > 0)
        d = st[ok, b] - st[ok, a]
        out[name] = [int(d.mean()), int(d.min()), int(np.percentile(d, 90)), int(d.max()), int(ok.sum())] \
            if ok.any() else None
    stat(0, 6, 'setup')           # start -> ring loop entry (item lookup, unit decode)
    stat(6, 7, 'first_kgroup')    # the first k-group's loads -> its MFMAs issued
    stat(0, 5, 'ring_fill')       # start -> 4th k-group consumed (units with >= D k-groups)
    stat(0, 1, 'main_loop')       # start -> k loop done
    stat(1, 2, 'lds_reduce')
    stat(2, 3, 'slab_ticket')
    stat(3, 4, 'last_finish')     # last arriver: slab sums + gradient RMW + clip partial
    stat(2, 4, 'direct_finish')   # single-chunk tiles (no stamp 3): gradient RMW
    stat(0, 4, 'total_last')
    stat(0, 3, 'total_nonlast')
    return out


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    res = {'rows': rows}
    critic = make(CRITIC, rows)
    res['critic'] = time_launch(critic, rows)
    res['critic_stamps'] = stamps(critic, rows)
    for name, shapes in (('actor', ACTOR), ('mult', MULT), ('256x256', [(256, 256)]), ('3x256x256', [(256, 256)] * 3),
                         ('256x16', [(256, SA)]), ('1x256', [(1, 256)])):
        it = make(shapes, rows)
        res[name] = time_launch(it, rows)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
