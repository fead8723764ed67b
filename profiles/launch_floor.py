"""Per-launch floor on the MI355X: back-to-back tiny kernels on one stream
(torch elementwise on 1 element, and a drpo row kernel on 4096 rows)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    import drpo_amd
    from drpo_amd import _lib
    L = _lib.lib()
    x = torch.zeros(1, device='cuda')
    print('torch add_ 1 elem: %.2f us/launch' % timeit(lambda: x.add_(1)))
    raw = torch.randn(4096, 1, device='cuda')
    lam = torch.empty(4096, device='cuda')
    s = _lib.stream()
    print('drpo_multiplier_out 4096: %.2f us/launch' % timeit(
        lambda: L.drpo_multiplier_out(4096, raw.data_ptr(), 50.0, lam.data_ptr(), s)))
    g = torch.randn(1 << 20, device='cuda')
    part = torch.empty(1024, device='cuda')
    print('drpo_grad_sumsq 1M: %.2f us/launch' % timeit(lambda: L.drpo_grad_sumsq(g.data_ptr(), g.numel(),
                                                                                   part.data_ptr(), s)))
    # graph-captured sequence of the same tiny kernels
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for _ in range(10):
            x.add_(1)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=st):
        for _ in range(100):
            x.add_(1)
    print('graph of 100 x add_: %.2f us/kernel' % (timeit(lambda: gr.replay(), n=50) / 100))


if __name__ == '__main__':
    main()
