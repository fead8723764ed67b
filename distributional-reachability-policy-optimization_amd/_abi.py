"""ctypes prototypes mirroring include/drpo_hip.h (keep the two in sync; the CPU test
suite checks every declared symbol is exported and every prototype here exists in
the header)."""
import ctypes

from ctypes import c_int, c_int64, c_uint64, c_float, c_size_t, c_void_p, c_char_p, POINTER

P = c_void_p


class RolloutDesc(ctypes.Structure):
    """drpo_rollout_desc_t"""
    _fields_ = [
        ('S', c_int), ('A', c_int), ('C', c_int), ('Ha', c_int), ('Hm', c_int), ('B', c_int), ('H', c_int),
        ('env_id', c_int), ('tracking_surr_start', c_int), ('tracking_n_surr', c_int),
        ('quad_x_threshold', c_float), ('quad_z_threshold', c_float),
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
    ]


# name -> (restype, argtypes)
PROTOTYPES = {
    'drpo_version': (c_int, []),
    'drpo_last_error': (c_char_p, []),
    'drpo_rollout_workspace_size': (c_size_t, [c_int, c_int, c_int]),
    'drpo_rollout_count_offset': (c_size_t, [c_int, c_int, c_int]),
    'drpo_rollout': (c_int, [POINTER(RolloutDesc), P]),
    'drpo_env_constraints': (c_int, [c_int, c_int, c_int, c_float, c_float, P, c_int64, c_int, P, P, P, P]),
    'drpo_sample_without_replacement': (c_int, [P, c_int64, c_int64, c_uint64, c_uint64, P]),
    'drpo_event_create': (c_int, [POINTER(c_void_p)]),
    'drpo_event_destroy': (c_int, [P]),
    'drpo_event_record': (c_int, [P, P]),
    'drpo_event_elapsed_ms': (c_int, [POINTER(c_float), P, P]),
    'drpo_grad_sumsq_blocks': (c_int, [c_int64]),
    'drpo_grad_sumsq': (c_int, [P, c_int64, P, P]),
    'drpo_adam': (c_int, [P, P, P, P, c_int64, c_float, c_float, c_float, c_float, c_float, c_float, P, c_int,
                          c_float, P, P]),
    'drpo_ema': (c_int, [P, P, c_int64, c_float, P]),
    'drpo_normalizer_workspace_size': (c_size_t, [c_int64, c_int]),
    'drpo_normalizer_fit': (c_int, [P, c_int64, c_int, P, P, P, P]),
    'drpo_normalize': (c_int, [P, P, P, c_float, P, c_int64, c_int, P]),
}


def declare(lib):
    for name, (res, args) in PROTOTYPES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
