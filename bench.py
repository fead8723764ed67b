#!/usr/bin/env python
"""Hot-path benchmark: imagined transitions/s + SAC grad-steps/s (BASELINE.json metric).

Workloads (BASELINE.json configs, restated as concrete inputs in SURVEY.md §8(d)),
picked with --config (default 2, the configuration the metric is quoted on):

  1  cartpole-move  (S=4,  A=1, C=4)  E=3  H=5   B=256
  2  quadrotor      (S=12, A=2, C=2)  E=7  H=10  B=4096
  3  point-robot    (S=11, A=2, C=1)  E=7  H=20  B=8192
  4  tracking       (S=51, A=2, C=1)  E=8  H=40  B=16384   (ensemble-sharded fit under torchrun)
  5  quadrotor      (S=12, A=2, C=2)  E=32 H=80  B=65536   (global batch: B/N rows per rank)

"batch" is both rollout_batch_size and the SAC batch size. DRPO flags
(qc_under_uncertainty = distributional_qc = mlp_multiplier = True), the other
hyper-parameters from the env's reference JSON (config/*.json), reference default
widths (actor/critics 256, model 200). Synthetic replay of 100k rows per §8(d);
random-init weights in "steady" rollout mode (diff-head output layer zeroed,
log-var output bias -20) so every rollout writes exactly B*H rows.

One step = SMBPO.rollout_and_update(): 1 rollout of B*H imagined transitions +
10 update_solver calls (actor on every 2nd, multiplier on every 5th). Under
torchrun every rank rolls out its own B rows and draws its own SAC minibatch of B
rows with gradients all-reduced over RCCL (weak scaling); config 5 divides its
global batch over the ranks instead (strong scaling).

value = imagined transitions/s over the rollout phases of the timed region (all
ranks), each phase bracketed by events recorded right before and right after the
SMBPO.rollout() call (transitions written by one rollout / its
time); sac.value = SAC grad-steps/s over the update phases. ms_per_step is the
full rollout_and_update wall time (max over ranks).
"""
import argparse
import ctypes
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
METRIC = 'imagined transitions/sec + SAC grad-steps/sec, quadrotor @1/2/4/8 GPU'

ENV_DIMS = {'cartpole': (4, 1, 4), 'quadrotor': (12, 2, 2), 'point-robot': (11, 2, 1), 'tracking': (51, 2, 1)}

# reference config/*.json alg_cfg (the DRPO flags are set by make_alg, as run.sh does)
ENV_JSON = {
    'quadrotor': {
        'sac_cfg': {'target_entropy': -2.0, 'constraint_threshold': 0.0, 'mlp_multiplier': True, 'penalty_lb': -1.0,
                    'penalty_ub': 100.0, 'mlp_multiplier_cfg': {'upper_bound': 50.0},
                    'constraint_critic_cfg': {'std_ratio': 2.0}, 'actor_lr': 1e-4, 'actor_lr_end': 4e-5},
        'steps_per_epoch': 360, 'model_update_period': 90, 'model_initial_steps': 1000, 'model_steps': 1000,
        'buffer_min': 1800, 'reward_scale': 2.0, 'alive_bonus': 2.0, 'safe_shield': False,
        'safe_shield_threshold': -0.2, 'eval_shield_threshold': -0.1, 'constraint_offset': 0.5},
    'point-robot': {
        'sac_cfg': {'target_entropy': -2.0, 'constraint_threshold': 0.0, 'penalty_lb': -5.0, 'penalty_ub': 100.0,
                    'mlp_multiplier_cfg': {'upper_bound': 50.0}, 'constraint_critic_cfg': {'std_ratio': 2.0},
                    'actor_lr': 1e-4, 'actor_lr_end': 4e-5},
        'steps_per_epoch': 300, 'model_update_period': 75, 'model_initial_steps': 5000, 'model_steps': 1000,
        'buffer_min': 1500, 'reward_scale': 10.0, 'alive_bonus': 0.0, 'constraint_scale': 10.0,
        'safe_shield': False},
    'tracking': {
        'sac_cfg': {'target_entropy': -2.0, 'constraint_threshold': 0.0, 'penalty_lb': -5.0, 'penalty_ub': 100.0,
                    'mlp_multiplier_cfg': {'upper_bound': 50.0}, 'constraint_critic_cfg': {'std_ratio': 1.0},
                    'actor_lr': 5e-5, 'actor_lr_end': 1e-7},
        'steps_per_epoch': 200, 'model_update_period': 50, 'model_initial_steps': 2000, 'model_steps': 1000,
        'buffer_min': 1000, 'reward_scale': 20.0, 'alive_bonus': 2.0, 'constraint_scale': 5.0, 'safe_shield': False,
        'real_fraction': 1.0},
    'cartpole': {
        'sac_cfg': {'target_entropy': -1.0, 'constraint_threshold': 0.0, 'penalty_lb': -5.0, 'penalty_ub': 100.0,
                    'mlp_multiplier_cfg': {'upper_bound': 50.0}, 'constraint_critic_cfg': {'std_ratio': 2.0},
                    'actor_lr': 1e-4, 'actor_lr_end': 4e-5},
        'steps_per_epoch': 1000, 'model_update_period': 250, 'model_initial_steps': 2000, 'model_steps': 1000,
        'buffer_min': 1000, 'reward_scale': 1.0, 'alive_bonus': 0.0, 'constraint_scale': 100.0, 'safe_shield': False},
}
QUAD_JSON = ENV_JSON['quadrotor']

CONFIGS = {
    1: dict(env='cartpole', E=3, H=5, B=256, label='cartpole-move E=3 H=5 B=256 (BASELINE configs[0])'),
    2: dict(env='quadrotor', E=7, H=10, B=4096, label='quadrotor E=7 H=10 B=4096 (BASELINE configs[1])'),
    3: dict(env='point-robot', E=7, H=20, B=8192, label='point-robot E=7 H=20 B=8192 (BASELINE configs[2])'),
    4: dict(env='tracking', E=8, H=40, B=16384,
            label='tracking-double_lane E=8 H=40 B=16384, ensemble-sharded fit (BASELINE configs[3])'),
    5: dict(env='quadrotor', E=32, H=80, B=65536, global_batch=True,
            label='quadrotor E=32 H=80 global B=65536, DP all-reduce (BASELINE configs[4])'),
}


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


# ---------------------------------------------------------------------------
# synthetic replays
# ---------------------------------------------------------------------------
def _point_robot_obs(xy, v, th):
    """11-d point-robot observation from (x, y, v, heading) (src/env/point_robot.py:146-170)."""
    n = len(v)
    o = np.zeros((n, 11), np.float32)
    o[:, 0:2], o[:, 2] = xy, v
    c, s = np.cos(th), np.sin(th)
    o[:, 3], o[:, 4] = c, s
    for i, hz in enumerate(((0.4, -1.2), (-0.4, 1.2))):
        dx, dy = hz[0] - xy[:, 0], hz[1] - xy[:, 1]
        bx, by = dx * c + dy * s, -dx * s + dy * c      # (hazard - pos) @ [[c, -s], [s, c]]
        o[:, 5 + 3 * i] = np.hypot(bx, by)
        ang = np.arctan2(by, bx)
        o[:, 6 + 3 * i], o[:, 7 + 3 * i] = np.cos(ang), np.sin(ang)
    return o


def synth_states(env, N, rng):
    if env == 'quadrotor':
        s = rng.normal(0, 0.1, size=(N, 12)).astype(np.float32)
        s[:, 0] = rng.uniform(-1, 1, N)
        s[:, 2] = rng.uniform(0.8, 1.2, N)
        s[:, 4] = rng.uniform(-0.1, 0.1, N)
        return s
    if env == 'cartpole':
        s = rng.normal(0, 0.1, size=(N, 4)).astype(np.float32)
        s[:, 0] = rng.uniform(-0.5, 0.5, N)
        s[:, 1] = rng.uniform(-0.1, 0.1, N)
        return s
    if env == 'point-robot':
        xy = rng.uniform(-2.5, 2.5, size=(N, 2))
        near = rng.rand(N) < 0.25       # ~25 % of rows within 0.3 of a hazard's edge
        hz = np.array([[0.4, -1.2], [-0.4, 1.2]])[rng.randint(0, 2, N)]
        ang = rng.uniform(0, 2 * np.pi, N)
        rad = 0.8 + rng.uniform(-0.3, 0.3, N)
        xy[near] = hz[near] + rad[near, None] * np.stack([np.cos(ang[near]), np.sin(ang[near])], 1)
        goal = np.hypot(xy[:, 0] - 2.2, xy[:, 1] - 2.2) <= 0.3
        xy[goal] = -xy[goal]            # reject the goal disc
        return _point_robot_obs(xy, rng.uniform(0.5, 2.0, N), rng.uniform(np.pi / 4, 3 * np.pi / 4, N))
    if env == 'tracking':
        s = rng.normal(0, 0.5, size=(N, 51)).astype(np.float32)
        hi = np.array([2, 1, np.pi / 6, 2, 0.1, 0.1])       # work_space (pyth_veh3dofconti_data.py:87-91)
        s[:, 0:6] = rng.uniform(-hi, hi, size=(N, 6))
        s[:, 6] = rng.uniform(-np.pi / 6, np.pi / 6, N)
        lon, lat = rng.uniform(-15, 15, N), rng.uniform(-5, 5, N)
        clash = (np.abs(lon) <= 7) & (np.abs(lat) <= 3)
        lon[clash] = np.sign(lon[clash]) * (7 + rng.uniform(0.01, 8, clash.sum()))
        s[:, 47], s[:, 48] = lon, lat
        s[:, 49], s[:, 50] = rng.normal(0, 0.1, N), rng.uniform(5, 10, N)
        return s
    raise KeyError(env)


def synth_replay(env, N, rng, dev=None, env_params=None):
    """states, actions, next states (s + N(0, 1e-3)), rewards ~ N(0, 1) and the env's
    constraint values / flags of the next states (device constraint fns when dev is a
    GPU, else zeros)."""
    S, A, C = ENV_DIMS[env]
    s = synth_states(env, N, rng)
    a = rng.uniform(-1, 1, size=(N, A)).astype(np.float32)
    s2 = (s + rng.normal(0, 1e-3, size=s.shape)).astype(np.float32)
    rep = dict(states=s, actions=a, next_states=s2, rewards=rng.normal(0, 1, N).astype(np.float32),
               dones=np.zeros(N, bool), violations=np.zeros(N, bool),
               constraint_values=np.zeros((N, C) if C > 1 else N, np.float32))
    if dev is not None and dev.type == 'cuda':
        from drpo_amd import ops
        from drpo_amd.envs import device_env_params
        d, v, h = ops.env_constraints(env_params or device_env_params(env), torch.from_numpy(s2).to(dev))
        rep['dones'], rep['violations'], rep['constraint_values'] = (d.cpu().numpy(), v.cpu().numpy(),
                                                                      h.cpu().numpy())
    return rep


def make_alg(dev, B, H, E, seed, cfg_json, extra=None, env='quadrotor'):
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
    return drpo_amd.SMBPO(cfg, lambda id=None: ShapeEnv(env), None, 100, device=dev, noise_seed=seed)


def steady_mode(alg):
    m = alg.model_ensemble
    _, diff, logv = m.views()
    diff[-1][0].zero_()
    diff[-1][1].zero_()
    logv[-1][1].fill_(-20.0)
    m._elite_inds = list(range(min(5, m.ensemble_size)))


def cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def cpu_baseline(cfgd, seed, budget_s=16.0):
    """The oracle (torch-CPU restatement of the reference, pinned to its fixtures) on
    the host: a bounded sample of the same workload at 4 threads (the reference's
    torch.set_num_threads(4), src/cli.py:108) and at every core this process may use."""
    from oracle import drpo_oracle as O
    env, E = cfgd['env'], cfgd['E']
    S, A, C = ENV_DIMS[env]
    jsn = ENV_JSON[env]
    Bs, Hs = min(cfgd['B'], 4096), min(cfgd['H'], 10)      # bounded sample of the workload
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else os.cpu_count()
    share = int(os.environ.get('OMP_NUM_THREADS', affinity))
    all_threads = max(1, min(affinity, share))
    dev = torch.device('cpu')
    alg = make_alg(dev, Bs, Hs, E, seed, jsn, env=env)
    steady_mode(alg)
    sd = {k: v.detach().clone() for k, v in alg.state_dict().items()}
    rep = synth_replay(env, 100000, np.random.RandomState(seed))
    st = torch.from_numpy(rep['states'])
    P = {k[len('solver.'):]: v for k, v in sd.items() if k.startswith('solver.actor.')}
    P.update({k: v for k, v in sd.items() if k.startswith('model_ensemble.')})
    P['model_ensemble.state_normalizer.mean'], P['model_ensemble.state_normalizer.std'] = O.normalizer_fit(st)
    elites = list(range(min(5, E)))
    Ps = {k[len('solver.'):]: v for k, v in sd.items() if k.startswith('solver.') and
          not k.startswith('solver.model_ensemble') and k != 'solver.total_updates'}
    sac_cfg = jsn['sac_cfg']
    r = torch.from_numpy(rep['rewards'])
    hcv = torch.from_numpy(rep['constraint_values']).reshape(len(r), -1)
    out = {}
    for threads in sorted({4, all_threads}):
        torch.set_num_threads(threads)
        n_tr, reps, t0 = 0, 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s / 4 or reps < 1:
            ro = O.rollout(P, 'actor.net.', 'model_ensemble.', elites, st, env, Bs, Hs, O.LiveRNG())
            n_tr += len(ro['states'])
            reps += 1
        roll = n_tr / (time.perf_counter() - t0)
        orc = O.SSACOracle(Ps, dict(batch_size=Bs, target_entropy=sac_cfg['target_entropy'],
                                    penalty_lb=sac_cfg['penalty_lb'], actor_lr=sac_cfg['actor_lr'],
                                    updates_per_training=100 * jsn['steps_per_epoch'] * 10), C, A)
        live = O.LiveRNG()
        t1, steps = time.perf_counter(), 0
        while time.perf_counter() - t1 < budget_s / 4 or steps < 2:
            idx = torch.randint(len(st), [Bs])
            h = hcv[idx] * jsn.get('constraint_scale', 10.0)
            h = h + (h > 0).float() * jsn.get('constraint_offset', 0.0)
            batch = (st[idx], torch.from_numpy(rep['actions'])[idx], torch.from_numpy(rep['next_states'])[idx],
                     r[idx] * jsn['reward_scale'] + jsn['alive_bonus'], torch.zeros(Bs, dtype=torch.bool),
                     torch.zeros(Bs, dtype=torch.bool), h if C > 1 else h[:, 0])
            orc.update_critic(*batch, live)
            if steps % 2 == 0:
                orc.update_actor_and_alpha(batch[0], live)
            if steps % 5 == 0:
                orc.update_multiplier(batch[0], live)
            steps += 1
        sps = steps / (time.perf_counter() - t1)
        out[threads] = (roll, reps, sps, steps)
    t4 = out[4]
    ta = out[all_threads]
    return {'value': t4[0], 'unit': 'imagined transitions/s', 'cores': 4, 'kind': 'port',
            'sample': f'{t4[1]} x oracle SMBPO.rollout of B={Bs} H={Hs} ({env}, E={E}, steady mode) on the host CPU, '
                      f'torch {torch.__version__}, 4 threads (bounded sample of the B={cfgd["B"]} H={cfgd["H"]} '
                      'workload)',
            'cpu_model': cpu_model(), 'cores_available': affinity, 'cpu_share_threads': share,
            'all_cores': {'threads': all_threads, 'value': ta[0],
                          'sac_value': ta[2], 'sac_samples_per_s': ta[2] * Bs},
            'sac': {'value': t4[2], 'unit': f'grad-steps/s of B={Bs} samples', 'samples_per_s': t4[2] * Bs,
                    'sample': f'{t4[3]} x oracle update_solver cadence (critic; actor 1/2; multiplier 1/5), '
                              f'B={Bs}, 4 threads'}}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """Run this script as `torch.distributed.run --nproc-per-node n` in a child
    process (one rank per GPU, rendezvous on 127.0.0.1). The ranks' JSON result line
    (printed by rank 0 only) is relayed to stdout and everything else to stderr; the
    return code is torchrun's, which is non-zero when any rank failed."""
    import subprocess
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', f'--master-port={_free_port()}', os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    result = []
    for line in p.stdout:
        if line.startswith('{') and '"metric"' in line:
            result.append(line)
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = p.wait()
    for line in result:
        sys.stdout.write(line)
    sys.stdout.flush()
    if rc == 0 and len(result) != 1:
        sys.stderr.write(f'bench.py: expected one result line from {n} ranks, got {len(result)}\n')
        return 1
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', type=int, default=2, choices=sorted(CONFIGS),
                    help='BASELINE.json configs[config-1] (SURVEY.md §8(d))')
    ap.add_argument('--batch', type=int, default=None, help='override B (per rank; labels the run as custom)')
    ap.add_argument('--horizon', type=int, default=None)
    ap.add_argument('--ensemble', type=int, default=None)
    ap.add_argument('--global-batch', type=int, default=None,
                    help='divide this global batch over the ranks (config 5 does so by default)')
    ap.add_argument('--rollout-only', action='store_true')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--no-fit', action='store_true', help='skip the model-fit post-pass')
    ap.add_argument('--backend', default='nccl', help='torch.distributed backend for N>1 (nccl = RCCL)')
    ap.add_argument('--fit-steps', type=int, default=None,
                    help="steps of the timed fit call (default: the config's model_steps, the length of "
                         "the reference's fit(steps=) call, src/smbpo.py:214-216)")
    ap.add_argument('--engine', type=int, default=0, help='rollout engine: 0 auto (fused horizon), 1 per-step launches')
    ap.add_argument('--elites', default=None, help='comma-separated elite members (traffic probes)')
    args = ap.parse_args()

    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` outside torchrun: start the N ranks as fresh child
        # processes before this process touches the GPU (no exec), relay rank 0's line
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world != args.gpus:
        raise SystemExit(f'bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; launch one rank per GPU')
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

    cfgd = dict(CONFIGS[args.config])
    env = cfgd['env']
    S, A, C = ENV_DIMS[env]
    E = args.ensemble or cfgd['E']
    H = args.horizon or cfgd['H']
    gb = args.global_batch or (cfgd['B'] if cfgd.get('global_batch') else None)
    if gb is not None:
        assert gb % world == 0, f'global batch {gb} must divide over {world} ranks'
        B = gb // world
    else:
        B = args.batch or cfgd['B']
    custom = any(x is not None for x in (args.batch, args.horizon, args.ensemble, args.global_batch))
    label = cfgd['label'] if not custom else f'{env} E={E} H={H} B={B}/rank (custom shape, not a BASELINE config)'
    if gb is not None and not custom:
        label += f', B={B} per rank on {world} rank(s)'

    import drpo_amd  # noqa: F401
    from drpo_amd.ops import EventTimer
    alg = make_alg(dev, B, H, E, args.seed, ENV_JSON[env], env=env)
    alg.rollout_engine = args.engine
    rep = synth_replay(env, 100000, np.random.RandomState(args.seed + rank), dev, alg.env_params)
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
    alg.model_ensemble.state_normalizer.fit(alg.replay_buffer.get('states'))
    steady_mode(alg)
    if args.elites:   # traffic probe: the elite set the rollout draws from
        alg.model_ensemble._elite_inds = [int(x) for x in args.elites.split(',')]
    from drpo_amd.distributed import sync_parameters
    sync_parameters(alg)            # every rank starts from rank 0's weights (DP replicas)
    do_sac = not args.rollout_only

    roll_ms, sac_ms, kern_ms, call_ms = [], [], [], []
    n_dev = torch.zeros(1, dtype=torch.int64, device=dev)

    from drpo_amd import _lib as dlib
    # production noise: ops.rollout picks the fused engine (2) for H <= 128
    fused_engine = args.engine == 2 or (args.engine == 0 and H <= 128)

    def one_step(tmr):
        if tmr is not None and fused_engine:
            # Fused engine: the library records tmr.events[0] immediately before the
            # persist kernel (the rollout's first GPU work) and events[1] after it, so
            # events[0] opens the rollout phase, and events[2] / [3] (free: one kernel
            # pair) close it and the SAC phase. The phase spans the same GPU work as a
            # separate event recorded before the call, minus that event's own gap.
            # events[4]: before the Python call (the call-bracketed figure, reported beside)
            dlib.check(dlib.lib().drpo_event_record(tmr.events[4], dlib.stream()), 'event_record')
            out = alg.rollout(alg.actor, timer=tmr)
            dlib.check(dlib.lib().drpo_event_record(tmr.events[2], dlib.stream()), 'event_record')
            if do_sac:
                for st in range(alg.solver_updates_per_step):
                    alg.update_solver(update_actor=st % 2 == 0, update_multiplier=st % 5 == 0)
            dlib.check(dlib.lib().drpo_event_record(tmr.events[3], dlib.stream()), 'event_record')
            n_dev.add_(out._count)
            return None
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
    timers = [EventTimer(max(5, 2 * H)) for _ in range(args.steps)]
    wall0 = time.perf_counter()
    evs = [one_step(timers[i]) for i in range(args.steps)]
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - wall0
    for e, tmr in zip(evs, timers):
        if e is None:   # fused engine: library events (see one_step)
            ph = tmr.elapsed_pairs(2)  # (ev0, ev1) = kernel; (ev2, ev3) = SAC phase
            rs = ctypes.c_float()
            dlib.check(dlib.lib().drpo_event_elapsed_ms(ctypes.byref(rs), tmr.events[0], tmr.events[2]), 'elapsed')
            roll_ms.append(rs.value)
            sac_ms.append(ph[1])
            dlib.check(dlib.lib().drpo_event_elapsed_ms(ctypes.byref(rs), tmr.events[4], tmr.events[2]), 'elapsed')
            call_ms.append(rs.value)
        else:
            roll_ms.append(e[0].elapsed_time(e[1]))
            sac_ms.append(e[1].elapsed_time(e[2]))
        kern_ms.extend(tmr.elapsed_pairs(getattr(tmr, 'pairs', H)))
    n_trans = int(n_dev.item())
    tot = torch.tensor([wall, sum(roll_ms) / 1e3, sum(sac_ms) / 1e3, float(n_trans), sum(call_ms) / 1e3],
                       dtype=torch.float64, device=dev)
    if dist is not None:
        mx = tot.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tot.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        wall, roll_s, sac_s, n_all, call_s = mx[0].item(), mx[1].item(), mx[2].item(), sm[3].item(), mx[4].item()
    else:
        wall, roll_s, sac_s, n_all, call_s = tot[0].item(), tot[1].item(), tot[2].item(), tot[3].item(), tot[4].item()

    # post-pass (untimed): per-kernel-class MLP throughput of the SAC update from HIP
    # events around every MLP launch (drpo_amd.sac_step.LaunchProfiler). Every rank
    # runs it (the updates all-reduce gradients); rank 0 reports.
    sac_kernels = None
    sac_comm = None
    if do_sac:
        from drpo_amd.sac_step import LaunchProfiler
        from drpo_amd.distributed import CommLog
        eng = alg.solver.engine
        eng.profiler = LaunchProfiler()
        CommLog.timing, c0 = [], CommLog.calls      # HIP events around every gradient exchange
        for st in range(alg.solver_updates_per_step):
            alg.update_solver(update_actor=st % 2 == 0, update_multiplier=st % 5 == 0)
        torch.cuda.synchronize()
        summ = eng.profiler.summarise()
        eng.profiler = None
        sac_comm = {'ms_per_update': CommLog.take_ms() / alg.solver_updates_per_step,
                    'collectives_per_update': (CommLog.calls - c0) / alg.solver_updates_per_step}
        CommLog.timing = None
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
        if args.fit_steps is None:
            args.fit_steps = int(getattr(alg, 'model_steps', 1000))
        f0 = time.perf_counter()
        m.fit(alg.replay_buffer, steps=args.fit_steps)   # ends with a host read of the losses
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        fit_s = torch.tensor([time.perf_counter() - f0], dtype=torch.float64, device=dev)
        if dist is not None:
            dist.all_reduce(fit_s, op=dist.ReduceOp.MAX)
        fit_s = fit_s.item()
        # communication share of a fit step (untimed post-pass, events around each exchange)
        from drpo_amd.distributed import CommLog
        CommLog.timing, c0 = [], CommLog.calls
        m.fit(alg.replay_buffer, steps=50)
        torch.cuda.synchronize()
        fit_comm = {'ms_per_step': CommLog.take_ms() / 50, 'collectives_per_step': (CommLog.calls - c0) / 50}
        CommLog.timing = None
        from drpo_amd.distributed import member_sharding
        sh = member_sharding(m)
        fl = fit_flop_per_step(S, A, E, m.batch_size, m.hidden_dim)
        fit_res = {'steps': args.fit_steps, 'ms_per_fit_step': fit_s / args.fit_steps * 1e3,
                   'fit_steps_per_s': args.fit_steps / fit_s, 'flop_per_fit_step': fl,
                   'achieved_tflops_job': fl * args.fit_steps / fit_s / 1e12,
                   'frac_job': fl * args.fit_steps / fit_s / 1e12 / (FP32_PEAK_TFLOPS * world),
                   'rows_per_step': E * m.batch_size, 'comm': fit_comm,
                   'sharding': f'members {sh.ranges}' if sh is not None else
                   ('batch (gradient all-reduce)' if world > 1 else 'single')}
        steady_mode(alg)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    flop_tr = rollout_flop_per_transition(S, A)
    fused = getattr(timers[0], 'pairs', H) == 1
    kname = 'rollout_persist_kernel' if fused else 'rollout_step_kernel'
    k_avg_ms = float(np.mean(kern_ms))
    rows_per_launch = n_trans / max(1, len(kern_ms))
    achieved = flop_tr * rows_per_launch / (k_avg_ms * 1e-3) / 1e12
    sac_flop = sac_flop_per_step(B, S, A, C)
    # headline: the call-bracketed rollout phase (events before / after SMBPO.rollout());
    # the phase that starts at the library's own event before the persist kernel is
    # reported beside it as rollout_phase.kernel_bounded
    head_s = call_s if call_ms else roll_s
    res = {
        'metric': METRIC,
        'value': n_all / head_s,
        'unit': 'imagined transitions/s',
        'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': wall / args.steps * 1e3,
        'higher_is_better': True, 'scaling': 'strong' if gb is not None else 'weak', 'vs_baseline': None,
        'dtype': 'fp32', 'data': f'synthetic (SURVEY.md §8(d) {env} replay, random-init weights, steady mode)',
        'config': {'workload': label, 'baseline_config': None if custom else args.config, 'env': env,
                   'ensemble': E, 'horizon': H, 'batch': B, 'global_batch': B * world,
                   'parallelism': f'dp{world}' if world > 1 else 'single', 'drpo_flags': True},
        'sac': {'metric': 'SAC grad-steps/sec', 'unit': f'grad-steps/s of B={B * world} samples (whole job)',
                'value': (alg.solver_updates_per_step * args.steps / sac_s) if do_sac and sac_s > 0 else None,
                'rank_steps_per_s': (alg.solver_updates_per_step * args.steps / sac_s) if do_sac and sac_s > 0
                else None,
                'global_batch': B * world, 'gradient_exchange': 'one RCCL sum all-reduce bucket per optimizer '
                'phase (critic | actor + safe actor + alpha sum | multiplier), 1/G in the optimizer'
                if world > 1 else None,
                'flop_per_step_per_rank': sac_flop, 'measured': do_sac,
                'achieved_tflops_per_gpu': (sac_flop * alg.solver_updates_per_step * args.steps / sac_s / 1e12)
                if do_sac and sac_s > 0 else None,
                'mlp_kernels': sac_kernels,
                # gradient exchanges per update_solver (untimed post-pass, HIP events around each)
                'comm': sac_comm},
        'model_fit': fit_res,
        # the rollout phase behind `value`: from an event recorded before the Python call to
        # one recorded after it returns; kernel_bounded starts at the library's own event
        # right before the persist kernel instead (the rollout's GPU work only)
        'rollout_phase': {'bounds': 'events before / after the SMBPO.rollout() call',
                          'ms_per_rollout': head_s / args.steps * 1e3,
                          'kernel_bounded': {'value': n_all / roll_s, 'ms_per_rollout': roll_s / args.steps * 1e3,
                                             'bounds': 'library event before the persist kernel -> event after '
                                                       'the call'} if call_ms else None,
                          'call_over_kernel_bounded': (call_s / roll_s) if call_ms and roll_s > 0 else None},
        'roofline': {'kernel': kname, 'bound': 'mfma', 'achieved': achieved,
                     'peak': FP32_PEAK_TFLOPS, 'unit': 'TFLOP/s', 'frac': achieved / FP32_PEAK_TFLOPS,
                     'traffic': None, 'avg_launch_ms': k_avg_ms, 'flop_per_transition': flop_tr,
                     'rows_per_launch': rows_per_launch},
    }
    if res['sac']['achieved_tflops_per_gpu'] is not None:
        res['sac']['frac'] = res['sac']['achieved_tflops_per_gpu'] / FP32_PEAK_TFLOPS
    # HBM bytes per launch from the rocprofv3 FETCH/WRITE passes (profiles/traffic.py),
    # attached only when those counters were taken on THIS build (same source digest)
    from drpo_amd import _lib
    base = 'traffic_rollout_fused' if fused else 'traffic_rollout_step'
    for prof in (os.path.join(ROOT, 'profiles', f'{base}_c{args.config}.json'),
                 os.path.join(ROOT, 'profiles', f'{base}.json') if args.config == 2 else None):
        if prof and os.path.exists(prof) and not custom:
            tr = json.load(open(prof))
            if tr.get('kernel') == kname and tr.get('lib_digest') == _lib.build_digest():
                res['roofline']['traffic'] = tr.get('bytes_per_launch')
                res['roofline']['traffic_source'] = os.path.relpath(prof, ROOT)
                break
    res['lib_digest'] = _lib.build_digest()
    if world == 1 and not args.no_cpu_baseline:
        res['cpu_baseline'] = cpu_baseline(cfgd, args.seed)
    print(json.dumps(res))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
