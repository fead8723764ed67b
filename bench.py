#!/usr/bin/env python
"""Hot-path benchmark: imagined transitions/s + SAC grad-steps/s (BASELINE.json metric).

Workload (BASELINE.json configs[1]): quadrotor (S=12, A=2, C=2), ensemble E=7,
horizon H=10, batch B=4096 (rollout_batch_size = sac batch_size = B), DRPO flags
(qc_under_uncertainty = distributional_qc = mlp_multiplier = True), reference
default widths (actor/critics 256, model 200). Synthetic replay of 100k rows per
SURVEY.md §8(d); random-init weights in "steady" rollout mode (diff-head output
layer zeroed, log-var output bias -20) so every rollout writes exactly B*H rows.

One step = SMBPO.rollout_and_update(): 1 rollout of B*H imagined transitions +
10 update_solver calls (actor on every 2nd, multiplier on every 5th). With
--gpus N (torchrun), each rank runs its own rollout shard of B rows and its own
SAC minibatch of B rows with gradients all-reduced over RCCL (weak scaling).

value = imagined transitions/s over the rollout phases of the timed region (all
ranks); sac.value = SAC grad-steps/s over the update phases. ms_per_step is the
full rollout_and_update wall time (max over ranks).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_PEAK_TFLOPS = 157.3   # MI355X dense fp32 (matrix == vector rate), /opt/skills/guides/MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0


def rollout_flop_per_transition(S, A, Ha=256, Hm=200):
    # 2 * MACs of actor (S->Ha->Ha->2A) + member (S+A->Hm->Hm, 2 x (Hm->Hm->S+1))
    return 2 * ((S * Ha + Ha * Ha + Ha * 2 * A) + ((S + A) * Hm + 3 * Hm * Hm + 2 * Hm * (S + 1)))


def sac_flop_per_step(B, S=12, A=2, C=2, H=256):
    """per-sample MACs of one update_solver at the rollout_and_update
    cadence (critic every step, actor 1/2, multiplier 1/5), backward = 2x forward."""
    Fpi = S * H + H * H + H * 2 * A
    Fq = (S + A) * H + H * H + H
    Fqc = (S + A) * H + H * H + 2 * (H * H + H * C)
    Fqcm = (S + A) * H + H * H + H * H + H * C
    Fl = (S + 1) * H + H * H + H
    critic = 2 * Fpi + 8 * Fq + 4 * Fqc + Fqcm
    actor = 7 * Fpi + 3 * Fq + 7 * Fqc + Fl
    mult = 2 * Fpi + 2 * Fqc + 3 * Fl
    return 2 * B * (critic + actor / 2 + mult / 5)


def fit_flop_per_step(S, A, E, b, Hm=200):
    """one fit step = forward + backward (2x) over E*b rows of the
    member MLP (trunk + both heads): 3 x 2 x MACs."""
    mac = (S + A) * Hm + Hm * Hm + 2 * (Hm * Hm + Hm * (S + 1))
    return 3 * 2 * mac * E * b


def synth_replay(S, A, C, N, rng):
    s = rng.normal(0, 0.1, size=(N, S)).astype(np.float32)
    s[:, 0] = rng.uniform(-1, 1, N)
    s[:, 2] = rng.uniform(0.8, 1.2, N)
    s[:, 4] = rng.uniform(-0.1, 0.1, N)
    a = rng.uniform(-1, 1, size=(N, A)).astype(np.float32)
    s2 = (s + rng.normal(0, 1e-3, size=s.shape)).astype(np.float32)
    h = np.stack([0.5 - s2[:, 2], s2[:, 2] - 1.5], 1).astype(np.float32)
    return dict(states=s, actions=a, next_states=s2, rewards=rng.normal(0, 1, N).astype(np.float32),
                dones=np.zeros(N, bool), violations=np.zeros(N, bool), constraint_values=h)


def make_alg(dev, B, H, E, seed, cfg_json, extra=None):
    import drpo_amd
    from drpo_amd.envs import ShapeEnv
    cfg = drpo_amd.SMBPO.Config()
    cfg.update(cfg_json)
    cfg.update({'horizon': H, 'rollout_batch_size': B, 'buffer_max': max(10 ** 6, B * H),
                'model_cfg': {'ensemble_size': E, 'num_elites': min(5, E)},
                'sac_cfg': {'batch_size': B, 'qc_under_uncertainty': True, 'distributional_qc': True,
                            'mlp_multiplier': True}})
    if extra:
        cfg.update(extra)
    drpo_amd.set_seed(seed)
    alg = drpo_amd.SMBPO(cfg, lambda id=None: ShapeEnv('quadrotor'), None, 100, device=dev, noise_seed=seed)
    return alg


QUAD_JSON = {  # reference config/quadrotor.json alg_cfg (DRPO flags set by make_alg, as run.sh does)
    'sac_cfg': {'target_entropy': -2.0, 'constraint_threshold': 0.0, 'mlp_multiplier': True, 'penalty_lb': -1.0,
                'penalty_ub': 100.0, 'mlp_multiplier_cfg': {'upper_bound': 50.0},
                'constraint_critic_cfg': {'std_ratio': 2.0}, 'actor_lr': 1e-4, 'actor_lr_end': 4e-5},
    'steps_per_epoch': 360, 'model_update_period': 90, 'model_initial_steps': 1000, 'model_steps': 1000,
    'buffer_min': 1800, 'reward_scale': 2.0, 'alive_bonus': 2.0, 'safe_shield': False,
    'safe_shield_threshold': -0.2, 'eval_shield_threshold': -0.1, 'constraint_offset': 0.5}


def steady_mode(alg):
    m = alg.model_ensemble
    _, diff, logv = m.views()
    diff[-1][0].zero_()
    diff[-1][1].zero_()
    logv[-1][1].fill_(-20.0)
    m._elite_inds = list(range(min(5, m.ensemble_size)))


def cpu_baseline(B, H, E, seed, budget_s=12.0):
    """Oracle (torch-CPU restatement of the reference) on the host: one bounded sample."""
    from oracle import drpo_oracle as O
    threads = 4                         # the reference's torch.set_num_threads(4) (src/cli.py:108)
    torch.set_num_threads(threads)
    dev = torch.device('cpu')
    import drpo_amd  # noqa: F401  (init replication only; no compute on CPU)
    alg = make_alg(dev, B, H, E, seed, QUAD_JSON)
    steady_mode(alg)
    sd = {k: v.detach().clone() for k, v in alg.state_dict().items()}
    rng = np.random.RandomState(seed)
    rep = synth_replay(12, 2, 2, 100000, rng)
    st = torch.from_numpy(rep['states'])
    P = {k[len('solver.'):]: v for k, v in sd.items() if k.startswith('solver.actor.')}
    P.update({k: v for k, v in sd.items() if k.startswith('model_ensemble.')})
    P['model_ensemble.state_normalizer.mean'], P['model_ensemble.state_normalizer.std'] = O.normalizer_fit(st)
    elites = list(range(min(5, E)))
    n_tr, t0 = 0, time.perf_counter()
    reps = 0
    while time.perf_counter() - t0 < budget_s / 2 or reps < 1:
        out = O.rollout(P, 'actor.net.', 'model_ensemble.', elites, st, 'quadrotor', B, H, O.LiveRNG())
        n_tr += len(out['states'])
        reps += 1
    roll_tps = n_tr / (time.perf_counter() - t0)
    # SAC: oracle update_critic / update_actor_and_alpha / update_multiplier at the
    # rollout_and_update cadence on batches drawn from the same synthetic replay
    Ps = {k[len('solver.'):]: v for k, v in sd.items() if k.startswith('solver.') and
          not k.startswith('solver.model_ensemble') and k != 'solver.total_updates'}
    orc = O.SSACOracle(Ps, dict(batch_size=B, target_entropy=-2.0, penalty_lb=-1.0, actor_lr=1e-4,
                                updates_per_training=100 * 360 * 10), 2, 2)
    live = O.LiveRNG()
    r = torch.from_numpy(rep['rewards'])
    hcv = torch.from_numpy(rep['constraint_values'])
    t1, steps = time.perf_counter(), 0
    while time.perf_counter() - t1 < budget_s / 2 or steps < 2:
        idx = torch.randint(len(st), [B])
        batch = (st[idx], torch.from_numpy(rep['actions'])[idx], torch.from_numpy(rep['next_states'])[idx],
                 r[idx] * 2.0 + 2.0, torch.zeros(B, dtype=torch.bool), torch.zeros(B, dtype=torch.bool),
                 hcv[idx] * 10.0 + (hcv[idx] > 0).float() * 0.5)
        orc.update_critic(*batch, live)
        if steps % 2 == 0:
            orc.update_actor_and_alpha(batch[0], live)
        if steps % 5 == 0:
            orc.update_multiplier(batch[0], live)
        steps += 1
    sac_sps = steps / (time.perf_counter() - t1)
    return {'value': roll_tps, 'unit': 'imagined transitions/s', 'cores': threads, 'kind': 'port',
            'sample': f'{reps} x oracle SMBPO.rollout (quadrotor B={B} H={H} E={E}, steady mode) on the host CPU '
                      f'(torch {torch.__version__}, {threads} threads)',
            'sac': {'value': sac_sps, 'unit': f'grad-steps/s of B={B} samples',
                    'sample': f'{steps} x oracle update_solver cadence (critic; actor 1/2; multiplier 1/5), '
                              f'B={B}, {threads} threads'}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=4096)
    ap.add_argument('--horizon', type=int, default=10)
    ap.add_argument('--ensemble', type=int, default=7)
    ap.add_argument('--rollout-only', action='store_true')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--no-fit', action='store_true', help='skip the model-fit post-pass')
    ap.add_argument('--backend', default='nccl', help='torch.distributed backend for N>1 (nccl = RCCL)')
    ap.add_argument('--fit-steps', type=int, default=50)
    ap.add_argument('--engine', type=int, default=0, help='rollout engine: 0 auto (fused horizon), 1 per-step launches')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    # --backend gloo + more ranks than GPUs: a rehearsal of the N>1 path on one box
    local = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(args.backend)
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    B, H, E = args.batch, args.horizon, args.ensemble

    import drpo_amd
    from drpo_amd.ops import EventTimer
    alg = make_alg(dev, B, H, E, args.seed + rank, QUAD_JSON)
    alg.rollout_engine = args.engine
    rep = synth_replay(12, 2, 2, 100000, np.random.RandomState(args.seed + rank))
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
    alg.model_ensemble.state_normalizer.fit(alg.replay_buffer.get('states'))
    steady_mode(alg)
    from drpo_amd.distributed import sync_parameters
    sync_parameters(alg)            # every rank starts from rank 0's weights (DP replicas)
    do_sac = not args.rollout_only
    if do_sac:
        try:
            alg.solver.engine   # noqa: B018
        except (ImportError, NotImplementedError):
            do_sac = False

    roll_ms, sac_ms, kern_ms, step_ms, n_trans = [], [], [], [], 0

    n_dev = torch.zeros(1, dtype=torch.int64, device=dev)

    def one_step(tmr):
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t2 = torch.cuda.Event(enable_timing=True)
        t0.record()
        out = alg.rollout(alg.actor, timer=tmr)
        t1.record()
        if do_sac:
            for st in range(alg.solver_updates_per_step):
                alg.update_solver(update_actor=st % 2 == 0, update_multiplier=st % 5 == 0)
        t2.record()
        n_dev.add_(out._count)            # device-side transition count (no host sync)
        return (t0, t1, t2)

    for _ in range(args.warmup):
        one_step(None)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    n_dev.zero_()
    # no host synchronisation inside the timed region: the host enqueues ahead of the
    # GPU, so the per-phase event intervals are GPU time, not host launch latency
    timers = [EventTimer(2 * H) for _ in range(args.steps)]
    wall0 = time.perf_counter()
    evs = [one_step(timers[i]) for i in range(args.steps)]
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - wall0
    for e, tmr in zip(evs, timers):
        roll_ms.append(e[0].elapsed_time(e[1]))
        sac_ms.append(e[1].elapsed_time(e[2]))
        kern_ms.extend(tmr.elapsed_pairs(getattr(tmr, 'pairs', H)))
    n_trans = int(n_dev.item())
    tot = torch.tensor([wall, sum(roll_ms) / 1e3, sum(sac_ms) / 1e3, float(n_trans)], dtype=torch.float64, device=dev)
    if dist is not None:
        mx = tot.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tot.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        wall, roll_s, sac_s, n_all = mx[0].item(), mx[1].item(), mx[2].item(), sm[3].item()
    else:
        wall, roll_s, sac_s, n_all = tot[0].item(), tot[1].item(), tot[2].item(), tot[3].item()

    # post-pass (untimed): per-kernel-class MLP throughput of the SAC update from HIP
    # events around every MLP launch (drpo_amd.sac_step.LaunchProfiler). Every rank
    # runs it (the updates all-reduce gradients); rank 0 reports.
    sac_kernels = None
    if do_sac:
        from drpo_amd.sac_step import LaunchProfiler
        eng = alg.solver.engine
        eng.profiler = LaunchProfiler()
        for st in range(alg.solver_updates_per_step):
            alg.update_solver(update_actor=st % 2 == 0, update_multiplier=st % 5 == 0)
        torch.cuda.synchronize()
        summ = eng.profiler.summarise()
        eng.profiler = None
        sac_kernels = {k: {'tflops': round(v['tflops'], 2), 'frac': round(v['tflops'] / FP32_PEAK_TFLOPS, 4),
                           'avg_launch_us': round(v['avg_ms'] * 1e3, 2), 'launches': v['launches']}
                       for k, v in summ.items() if ':' not in k}

    # model fit ("report the model-fit step time separately"): one
    # fit(steps=K) of the reference's E x 256-row steps on the synthetic replay; under
    # torchrun the members are sharded over the ranks (distributed.MemberShard)
    fit_res = None
    if not args.no_fit:
        m = alg.model_ensemble
        m.fit(alg.replay_buffer, steps=2)            # warm-up (workspaces, packing)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        f0 = time.perf_counter()
        m.fit(alg.replay_buffer, steps=args.fit_steps)   # ends with a host read of the losses
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        fit_s = torch.tensor([time.perf_counter() - f0], dtype=torch.float64, device=dev)
        if dist is not None:
            dist.all_reduce(fit_s, op=dist.ReduceOp.MAX)
        fit_s = fit_s.item()
        from drpo_amd.distributed import member_sharding
        sh = member_sharding(m)
        fl = fit_flop_per_step(12, 2, E, m.batch_size, m.hidden_dim)
        fit_res = {'steps': args.fit_steps, 'ms_per_fit_step': fit_s / args.fit_steps * 1e3,
                   'fit_steps_per_s': args.fit_steps / fit_s, 'flop_per_fit_step': fl,
                   'achieved_tflops_job': fl * args.fit_steps / fit_s / 1e12,
                   'rows_per_step': E * m.batch_size,
                   'sharding': f'members {sh.ranges}' if sh is not None else
                   ('batch (gradient all-reduce)' if world > 1 else 'single')}
        steady_mode(alg)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    flop_tr = rollout_flop_per_transition(12, 2)
    fused = getattr(timers[0], 'pairs', H) == 1
    kname = 'rollout_persist_kernel' if fused else 'rollout_step_kernel'
    k_avg_ms = float(np.mean(kern_ms))
    rows_per_launch = n_trans / max(1, len(kern_ms))
    achieved = flop_tr * rows_per_launch / (k_avg_ms * 1e-3) / 1e12
    res = {
        'metric': 'imagined transitions/sec + SAC grad-steps/sec, quadrotor @1/2/4/8 GPU',
        'value': n_all / roll_s,
        'unit': 'imagined transitions/s',
        'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': wall / args.steps * 1e3,
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': 'fp32', 'data': 'synthetic (SURVEY.md §8(d) quadrotor replay, random-init weights, steady mode)',
        'config': {'workload': 'quadrotor E=7 H=10 B=4096 (BASELINE configs[1])', 'env': 'quadrotor',
                   'ensemble': E, 'horizon': H, 'batch': B, 'global_batch': B * world,
                   'parallelism': f'dp{world}' if world > 1 else 'single', 'drpo_flags': True},
        'sac': {'metric': 'SAC grad-steps/sec', 'unit': f'grad-steps/s of B={B} samples (whole job)',
                'value': (alg.solver_updates_per_step * args.steps * world / sac_s) if do_sac and sac_s > 0 else None,
                'global_steps_per_s': (alg.solver_updates_per_step * args.steps / sac_s)
                if do_sac and sac_s > 0 else None,
                'global_batch': B * world, 'gradient_exchange': 'RCCL all-reduce (mean) per optimizer group'
                if world > 1 else None,
                'flop_per_step': sac_flop_per_step(B), 'measured': do_sac,
                'achieved_tflops_per_gpu': (sac_flop_per_step(B) * alg.solver_updates_per_step * args.steps / sac_s / 1e12)
                if do_sac and sac_s > 0 else None,
                'mlp_kernels': sac_kernels},
        'model_fit': fit_res,
        'roofline': {'kernel': kname, 'bound': 'mfma', 'achieved': achieved,
                     'peak': FP32_PEAK_TFLOPS, 'unit': 'TFLOP/s', 'frac': achieved / FP32_PEAK_TFLOPS,
                     'traffic': None, 'avg_launch_ms': k_avg_ms, 'flop_per_transition': flop_tr,
                     'rows_per_launch': rows_per_launch},
    }
    prof = os.path.join(ROOT, 'profiles', 'traffic_rollout_fused.json' if fused else 'traffic_rollout_step.json')
    if os.path.exists(prof):
        tr = json.load(open(prof))
        if tr.get('kernel') == kname:
            res['roofline']['traffic'] = tr.get('bytes_per_launch')
    if world == 1 and not args.no_cpu_baseline:
        res['cpu_baseline'] = cpu_baseline(B, H, E, args.seed)
    print(json.dumps(res))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
