"""Micro-benchmark of drpo_optim_step (csrc/optim.hip) on the config-2 parameter
groups (the model ensemble's fit step, the SAC critic group with its EMA target,
a scalar segment whose gradient is a sum of 256 partials), with and without the
packed-mirror refresh, clip and gradient zeroing: per-launch microseconds over
back-to-back launches (HIP events)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / reps, 2)


def main():
    import bench
    from drpo_amd.optim import fused_step, grad_sumsq
    dev = torch.device('cuda')
    cd = bench.CONFIGS[2]
    alg = bench.make_alg(dev, cd['B'], cd['H'], cd['E'], 0, bench.ENV_JSON[cd['env']], env=cd['env'])
    m = alg.model_ensemble
    g = m.group
    opt = m.optimizer
    sc = opt.step_scalars()
    res = {'fit_params': g.size}
    part = grad_sumsq(g.grad)

    def seg(**kw):
        return opt.segment(0, g.size, sc, **kw)
    variants = {
        'fit_product': dict(pack_map=g.pack_map(), zero_grad=True),
        'fit_no_map': dict(zero_grad=True),
        'fit_no_map_no_zero': dict(),
        'fit_clip_map': dict(clip=(part, 1.0), pack_map=g.pack_map(), zero_grad=True),
    }
    for name, kw in variants.items():
        s = [seg(**kw)]
        res[name] = timeit(lambda: fused_step(s))
    res['fit_sumsq'] = timeit(lambda: grad_sumsq(g.grad))
    sol = alg.solver
    cg, tg = sol.critic_group, sol.critic_target_group
    copt = sol.critic_optimizer
    csc = copt.step_scalars()
    cpart = grad_sumsq(cg.grad)
    res['critic_params'] = cg.size
    s = [copt.segment(0, cg.size, csc, clip=(cpart, 1.0), zero_grad=True, ema=(tg.data, 0.005),
                      pack_map=cg.pack_map(tg))]
    res['critic_product_like'] = timeit(lambda: fused_step(s))
    s = [copt.segment(0, cg.size, csc, zero_grad=True)]
    res['critic_adam_only'] = timeit(lambda: fused_step(s))
    aopt = sol.alpha_optimizer
    if aopt.tensor is None:
        aopt.tensor = sol.log_alpha.view(1)
    parts = torch.zeros(256, device=dev)
    s = [aopt.segment(0, 1, aopt.step_scalars(), grad=parts[:1], grad_from_sum=(parts, 4096, 256))]
    res['alpha_sum256'] = timeit(lambda: fused_step(s))
    s = [aopt.segment(0, 1, aopt.step_scalars(), grad=parts[:1], grad_from_sum=(parts, 4096, 1))]
    res['alpha_sum1'] = timeit(lambda: fused_step(s))
    print(json.dumps(res))


if __name__ == '__main__':
    main()
