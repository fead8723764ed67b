"""ctypes prototypes mirroring include/drpo_hip.h (keep the two in sync; the CPU test
suite checks every declared symbol is exported and every prototype here exists in
the header)."""
import ctypes

from ctypes import c_int, c_int64, c_uint64, c_float, c_double, c_size_t, c_void_p, c_char_p, POINTER

P = c_void_p


class RolloutDesc(ctypes.Structure):
    """drpo_rollout_desc_t"""
    _fields_ = [
        ('S', c_int), ('A', c_int), ('C', c_int), ('Ha', c_int), ('Hm', c_int), ('B', c_int), ('H', c_int),
        ('env_id', c_int), ('tracking_surr_start', c_int), ('tracking_n_surr', c_int),
        ('env_thr0', c_double), ('env_thr1', c_double),
        ('aW1', P), ('ab1', P), ('aW2', P), ('ab2', P), ('aW3', P), ('ab3', P),
        ('mW1', P), ('mb1', P), ('mW2', P), ('mb2', P), ('dW1', P), ('db1', P), ('dW2', P), ('db2', P),
        ('lW1', P), ('lb1', P), ('lW2', P), ('lb2', P),
        ('norm_mean', P), ('norm_std', P), ('min_lv', P), ('max_lv', P),
        ('members', POINTER(c_int)),
        ('replay_states', P), ('replay_ptr', c_int64), ('replay_cap', c_int64),
        ('init_idx', P), ('eps_a', P), ('eps_m', P),
        ('seed', c_uint64), ('ctr', c_uint64),
        ('vs', P), ('va', P), ('vs2', P), ('vr', P), ('vh', P), ('vd', P), ('vv', P),
        ('vptr', P), ('vcap', c_int64),
        ('workspace', P), ('rows_per_tile', c_int), ('step_events', POINTER(c_void_p)),
        ('engine', c_int), ('eps_layout', c_int),
    ]


class PackItem(ctypes.Structure):
    """drpo_pack_item_t"""
    _fields_ = [('W', P), ('P', P), ('PT', P), ('din', c_int), ('dout', c_int), ('nbatch', c_int),
                ('wstride', c_int64), ('pstride', c_int64), ('ptstride', c_int64)]


class PackMap(ctypes.Structure):
    """drpo_pack_map_t (lives in device memory)"""
    _fields_ = [('nlayers', c_int), ('off', c_int64 * 16), ('din', c_int * 16), ('dout', c_int * 16),
                ('nbatch', c_int * 16), ('poff', c_int64 * 16), ('P', P), ('PT', P), ('Pt', P)]


class OptimSeg(ctypes.Structure):
    """drpo_optim_seg_t"""
    _fields_ = [('p', P), ('g', P), ('m', P), ('v', P), ('start', c_int64), ('end', c_int64), ('adam', c_int),
                ('partial', P), ('n_partial', c_int), ('max_norm', c_float),
                ('lr_over_bc1', c_float), ('bc2_sqrt', c_float), ('beta1', c_float), ('beta2', c_float),
                ('eps', c_float), ('weight_decay', c_float), ('zero_grad', c_int),
                ('ema_target', P), ('ema_rate', c_float), ('ema_keep', c_float), ('map', P),
                ('grad_from_sum', P), ('grad_sum_rows', c_int64), ('grad_from_sum_kind', c_int),
                ('grad_scale', c_float), ('grad_sum_n', c_int), ('map_host', P)]


class EnsReduce(ctypes.Structure):
    """drpo_ens_reduce_t"""
    _fields_ = [('part', P), ('nbx', c_int), ('Z', c_int), ('S1', c_int), ('minlv', P), ('maxlv', P),
                ('weight', c_float), ('gscale', P), ('mse', P), ('loss', P), ('gmin', P), ('gmax', P)]


class EnsUpstream(ctypes.Structure):
    """drpo_ens_upstream_t"""
    _fields_ = [('D', P), ('LVR', P), ('s', P), ('s_zstride', c_int64), ('t', P), ('t_zstride', c_int64),
                ('b', c_int64), ('S', c_int), ('Z', c_int), ('minlv', P), ('maxlv', P), ('gscale', P), ('part', P)]


# name -> (restype, argtypes)
PROTOTYPES = {
    'drpo_version': (c_int, []),
    'drpo_last_error': (c_char_p, []),
    'drpo_build_digest': (c_char_p, []),
    'drpo_abi_sizeof': (c_int64, [c_char_p]),
    'drpo_rollout_workspace_size': (c_size_t, [c_int, c_int, c_int]),
    'drpo_rollout_count_offset': (c_size_t, [c_int, c_int, c_int]),
    'drpo_rollout': (c_int, [POINTER(RolloutDesc), P]),
    'drpo_env_constraints': (c_int, [c_int, c_int, c_int, c_double, c_double, P, c_int64, c_int, P, P, P, P]),
    'drpo_shield_mix': (c_int, [P, P, c_int64, c_int, c_int, P, P]),
    'drpo_shield_select': (c_int, [P, c_int, c_int64, c_int, c_int, c_int, c_float, P, P, P, P, P]),
    'drpo_sample_without_replacement': (c_int, [P, c_int64, c_int64, c_uint64, c_uint64, P]),
    'drpo_event_create': (c_int, [POINTER(c_void_p)]),
    'drpo_event_destroy': (c_int, [P]),
    'drpo_event_record': (c_int, [P, P]),
    'drpo_stream_wait_event': (c_int, [P, P]),
    'drpo_event_elapsed_ms': (c_int, [POINTER(c_float), P, P]),
    'drpo_grad_sumsq_blocks': (c_int, [c_int64]),
    'drpo_grad_sumsq': (c_int, [P, c_int64, P, P]),
    'drpo_adam': (c_int, [P, P, P, P, c_int64, c_float, c_float, c_float, c_float, c_float, c_float, P, c_int,
                          c_float, P, P]),
    'drpo_ema': (c_int, [P, P, c_int64, c_float, P]),
    'drpo_normalizer_workspace_size': (c_size_t, [c_int64, c_int]),
    'drpo_normalizer_fit': (c_int, [P, c_int64, c_int, P, P, P, P]),
    'drpo_normalize': (c_int, [P, P, P, c_float, P, c_int64, c_int, P]),
    'drpo_packed_size': (c_int64, [c_int, c_int]),
    'drpo_optim_step': (c_int, [POINTER(OptimSeg), c_int, P]),
    'drpo_grad_sumsq_multi': (c_int, [POINTER(c_void_p), POINTER(c_int64), POINTER(c_void_p), c_int, P]),
    'drpo_pack_weights': (c_int, [POINTER(PackItem), c_int, P]),
    'drpo_ens_gather': (c_int, [P, P, P, P, c_int64, P, c_int64, c_int64, P, c_uint64, c_uint64, c_int, c_int, P, P,
                                P, P]),
    'drpo_ens_gather_steps': (c_int, [P, P, P, P, c_int64, P, c_int64, c_int64, c_int64, P, c_uint64, c_uint64,
                                      c_int, c_int, P, P, P, P]),
    'drpo_ens_head': (c_int, [P, P, P, c_int64, c_int64, c_int, c_int, P, P, P, P, c_uint64, c_uint64, P, P, P, P,
                              P]),
    'drpo_ens_loss_workspace_size': (c_size_t, [c_int64, c_int, c_int]),
    'drpo_ens_loss': (c_int, [P, P, P, c_int64, P, c_int64, c_int64, c_int, c_int, P, P, c_float, P, P, P, P, P, P,
                              P, P, P]),
    'drpo_ens_loss_partials': (c_int, [P, P, P, c_int64, P, c_int64, c_int64, c_int, c_int, P, P, c_float, P, P, P,
                                       P, P, P, P, P, POINTER(EnsReduce), P]),
}


def declare(lib):
    for name, (res, args) in PROTOTYPES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args


class MlpLayer(ctypes.Structure):
    """drpo_mlp_layer_t"""
    _fields_ = [('W', P), ('b', P), ('din', c_int), ('dout', c_int), ('act', c_int), ('sy', P), ('sz', P),
                ('wstride', c_int64), ('bstride', c_int64)]


class MlpNet(ctypes.Structure):
    _fields_ = [('nl', c_int), ('L', MlpLayer * 3)]


class PolicyHead(ctypes.Structure):
    """drpo_policy_head_t"""
    _fields_ = [('mode', c_int), ('A', c_int), ('eps', P), ('site', ctypes.c_uint32), ('a', P), ('logp', P), ('u', P),
                ('e', P), ('amean', P)]


class MlpFwd(ctypes.Structure):
    """drpo_mlp_fwd_t"""
    _fields_ = [('src', P * 3), ('cols', c_int * 3), ('ld', c_int * 3), ('sstride', c_int64 * 3),
                ('nmean', P), ('nstd', P), ('save_x', P), ('net', MlpNet * 3), ('nnets', c_int), ('trunk', c_int),
                ('rows', c_int64), ('nbatch', c_int), ('head', PolicyHead), ('split_heads', c_int),
                ('ccb_out', P), ('ccb_dist', c_int), ('ccb_ratio', c_float), ('ccb_lmin', c_float), ('ccb_lmax', c_float),
                ('pair', c_int), ('head2', PolicyHead), ('pre', MlpNet), ('pre_head', PolicyHead),
                ('post', MlpNet), ('post_x', P)]


class MlpBwdLayer(ctypes.Structure):
    """drpo_mlp_bwd_layer_t"""
    _fields_ = [('W', P), ('din', c_int), ('dout', c_int), ('act', c_int), ('sy', P), ('sz', P), ('dz', P),
                ('wstride', c_int64), ('dz2', P)]


class MlpBwdNet(ctypes.Structure):
    _fields_ = [('nl', c_int), ('L', MlpBwdLayer * 3), ('gout', P), ('dx', P), ('dx_col0', c_int),
                ('dx_cols', c_int), ('dx_accumulate', c_int)]


class MlpBwd(ctypes.Structure):
    """drpo_mlp_bwd_t"""
    _fields_ = [('net', MlpBwdNet * 3), ('nnets', c_int), ('trunk', c_int), ('rows', c_int64), ('nbatch', c_int),
                ('split_heads', c_int), ('upstream', c_int)]


class WgradItem(ctypes.Structure):
    """drpo_wgrad_item_t"""
    _fields_ = [('dz', P), ('y', P), ('gW', P), ('gb', P), ('dout', c_int), ('din', c_int), ('rows', c_int64),
                ('zstride', c_int64), ('ystride', c_int64), ('gwstride', c_int64), ('gbstride', c_int64),
                ('nbatch', c_int), ('sq', P), ('sq_off', c_int), ('dz2', P)]


class BufferView(ctypes.Structure):
    """drpo_buffer_view_t"""
    _fields_ = [('s', P), ('a', P), ('s2', P), ('r', P), ('h', P), ('d', P), ('v', P), ('len', c_int64),
                ('ptr_dev', P), ('cap', c_int64)]


class ActorHead(ctypes.Structure):
    """drpo_actor_head_t"""
    _fields_ = [('B', c_int64), ('C', c_int), ('A', c_int), ('distributional', c_int), ('std_ratio', c_float),
                ('log_std_min', c_float), ('log_std_max', c_float), ('lams', P), ('lam_upper_bound', c_float),
                ('fixed_lam', c_float), ('clamp_lb', c_float), ('clamp_ub', c_float), ('u', P * 2), ('e', P * 2),
                ('dA', P * 2), ('dA2', P * 2), ('logp', P), ('log_alpha', P), ('lp_scale', c_float),
                ('target_entropy', c_float), ('alpha_sum', P)]


class CriticHead(ctypes.Structure):
    """drpo_critic_head_t"""
    _fields_ = [('B', c_int64), ('C', c_int), ('distributional', c_int), ('deterministic_backup', c_int),
                ('discount', c_float), ('qc_td_bound', c_float), ('lmin', c_float), ('lmax', c_float),
                ('log_alpha', P), ('r', P), ('h', P), ('d', P), ('dc', P), ('q0t', P), ('q1t', P), ('logp2', P),
                ('mu_t', P), ('ls_t', P), ('eps3', P), ('seed', c_uint64), ('ctr', c_uint64),
                ('q0', P), ('q1', P), ('mu', P), ('ls', P), ('dq0', P), ('dq1', P), ('dmu', P), ('dls', P),
                ('loss', P), ('loss_part', P), ('cost', c_int), ('v', P)]


class WgradAdam(ctypes.Structure):
    """drpo_wgrad_adam_t"""
    _fields_ = [('g', P), ('p', P), ('m', P), ('v', P), ('lr_over_bc1', c_float), ('bc2_sqrt', c_float),
                ('beta1', c_float), ('beta2', c_float), ('eps', c_float), ('weight_decay', c_float),
                ('map', P), ('map_host', P)]


class SumDesc(ctypes.Structure):
    """drpo_sum_t"""
    _fields_ = [('part', P), ('n', c_int), ('out', P)]


PROTOTYPES.update({
    'drpo_mlp_forward': (c_int, [POINTER(MlpFwd), P]),
    'drpo_mlp_forward_multi': (c_int, [POINTER(MlpFwd), P, c_int, c_uint64, c_uint64, P]),
    'drpo_mlp_backward_multi_head': (c_int, [POINTER(MlpBwd), P, c_int, POINTER(CriticHead), P]),
    'drpo_mlp_backward_multi_actor': (c_int, [POINTER(MlpBwd), P, c_int, POINTER(ActorHead), P]),
    'drpo_mlp_backward_multi': (c_int, [POINTER(MlpBwd), P, c_int, P]),
    'drpo_mlp_backward': (c_int, [POINTER(MlpBwd), P]),
    'drpo_mlp_backward_ens': (c_int, [POINTER(MlpBwd), POINTER(EnsUpstream), POINTER(EnsReduce), POINTER(EnsReduce),
                                      P]),
    'drpo_ens_fit_fb': (c_int, [POINTER(MlpFwd), POINTER(MlpBwd), POINTER(EnsUpstream), POINTER(EnsReduce),
                                POINTER(EnsReduce), P]),
    'drpo_mlp_wgrad_workspace_size': (c_size_t, [POINTER(WgradItem), c_int]),
    'drpo_mlp_wgrad_tiles': (c_int, [POINTER(WgradItem)]),
    'drpo_mlp_wgrad': (c_int, [POINTER(WgradItem), c_int, P, c_size_t, P]),
    'drpo_mlp_wgrad_reduce': (c_int, [POINTER(WgradItem), c_int, POINTER(EnsReduce), P, c_size_t, P]),
    'drpo_mlp_wgrad_sums': (c_int, [POINTER(WgradItem), c_int, POINTER(SumDesc), c_int, P, c_size_t, P]),
    'drpo_mlp_wgrad_adam': (c_int, [POINTER(WgradItem), c_int, P, POINTER(WgradAdam), P, c_size_t, P]),
    'drpo_ens_loss_reduce': (c_int, [POINTER(EnsReduce), P]),
    'drpo_sample_batch': (c_int, [POINTER(BufferView), POINTER(BufferView), c_int, c_int, c_int, c_int, c_int, P, P,
                                  c_uint64, c_uint64, c_float, c_float, c_float, c_float, P, P, P, P, P, P, P, P]),
    'drpo_policy_head': (c_int, [P, c_int64, c_int, c_int, P, c_uint64, c_uint64, ctypes.c_uint32, P, P, P, P, P,
                                 P]),
    'drpo_cc_dist': (c_int, [P, P, c_int64, c_int, c_float, c_float, c_float, P, c_uint64, c_uint64, P, P, P]),
    'drpo_cc_head': (c_int, [P, P, c_int64, c_int, c_int, c_float, c_float, c_float, P, P, P]),
    'drpo_critic_head': (c_int, [POINTER(CriticHead), P]),
    'drpo_actor_upstream': (c_int, [c_int64, c_int, c_int, c_float, c_float, c_float, P, P, P, P, P, P, P, P, P, P,
                                    c_float, c_float, c_float, c_float, P]),
    'drpo_squash_backward': (c_int, [c_int64, c_int, P, P, P, P, P, P, c_float, P, c_float, P, P, P]),
    'drpo_alpha_grad': (c_int, [P, P, c_int64, P, P]),
    'drpo_multiplier_head': (c_int, [c_int64, P, P, P, c_float, c_float, c_float, c_float, c_float, P, P, P]),
    'drpo_multiplier_out': (c_int, [c_int64, P, c_float, P, P]),
})
