// Library-wide C ABI: version, error reporting.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <stdlib.h>

#include "common.hpp"

static thread_local char g_err[1024] = "";

void drpo_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

DRPO_API const char* drpo_last_error(void) { return g_err; }

DRPO_API int drpo_version(void) { return 1; }

// HIP event helpers so hosts without a HIP binding (ctypes/cgo/JNI) can time
// individual kernels on the stream they run on. The events are timing-only: created
// without the system-scope release a default event record carries (measured: a
// default timing event left the GPU idle ~5.7 us per record between two kernels,
// profiles/r04a), since nothing reads memory through them.
DRPO_API int drpo_event_create(void** ev) {
  hipEvent_t e;
  hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  if (r != hipSuccess) {
    drpo_set_error("hipEventCreate: %s", hipGetErrorString(r));
    return DRPO_EHIP;
  }
  *ev = (void*)e;
  return DRPO_OK;
}

DRPO_API int drpo_event_destroy(void* ev) { return hipEventDestroy((hipEvent_t)ev) == hipSuccess ? DRPO_OK : DRPO_EHIP; }

DRPO_API int drpo_event_record(void* ev, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  return hipEventRecord((hipEvent_t)ev, stream) == hipSuccess ? DRPO_OK : DRPO_EHIP;
}

// stream waits for an event recorded on another stream of the same device (the model
// fit's side stream, ensemble_engine.fit): with the events above, the hand-off costs no
// system-scope fence
DRPO_API int drpo_stream_wait_event(drpo_stream_t stream_, void* ev) {
  const hipError_t r = hipStreamWaitEvent((hipStream_t)stream_, (hipEvent_t)ev, 0);
  if (r != hipSuccess) {
    drpo_set_error("hipStreamWaitEvent: %s", hipGetErrorString(r));
    return DRPO_EHIP;
  }
  return DRPO_OK;
}

DRPO_API int drpo_event_elapsed_ms(float* ms, void* start, void* stop) {
  hipError_t r = hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop);
  if (r != hipSuccess) {
    drpo_set_error("hipEventElapsedTime: %s", hipGetErrorString(r));
    return DRPO_EHIP;
  }
  return DRPO_OK;
}

// sizeof of every ABI struct by name (binding self-check: tests/test_abi.py compares
// these with the ctypes mirrors); -1 for an unknown name
DRPO_API int64_t drpo_abi_sizeof(const char* name) {
  struct E { const char* n; size_t s; };
  static const E table[] = {
      {"drpo_rollout_desc_t", sizeof(drpo_rollout_desc_t)}, {"drpo_mlp_layer_t", sizeof(drpo_mlp_layer_t)},
      {"drpo_mlp_net_t", sizeof(drpo_mlp_net_t)},           {"drpo_policy_head_t", sizeof(drpo_policy_head_t)},
      {"drpo_mlp_fwd_t", sizeof(drpo_mlp_fwd_t)},           {"drpo_mlp_bwd_layer_t", sizeof(drpo_mlp_bwd_layer_t)},
      {"drpo_mlp_bwd_net_t", sizeof(drpo_mlp_bwd_net_t)},   {"drpo_mlp_bwd_t", sizeof(drpo_mlp_bwd_t)},
      {"drpo_wgrad_item_t", sizeof(drpo_wgrad_item_t)},     {"drpo_buffer_view_t", sizeof(drpo_buffer_view_t)},
      {"drpo_critic_head_t", sizeof(drpo_critic_head_t)},   {"drpo_pack_item_t", sizeof(drpo_pack_item_t)},
      {"drpo_pack_map_t", sizeof(drpo_pack_map_t)},         {"drpo_optim_seg_t", sizeof(drpo_optim_seg_t)},
      {"drpo_ens_reduce_t", sizeof(drpo_ens_reduce_t)},
  };
  for (const E& e : table)
    if (strcmp(e.n, name) == 0) return (int64_t)e.s;
  return -1;
}
