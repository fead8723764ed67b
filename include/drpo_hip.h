/*
 * drpo_hip.h -- C ABI of libdrpo_hip.so, the MI355X (gfx950) hot path of
 * Distributional Reachability Policy Optimization.
 *
 * The reference (ManUtdMoon/Distributional-Reachability-Policy-Optimization) is
 * pure Python/PyTorch with no FFI; these entry points are what a binding for its
 * hot path binds (the Python package drpo_amd binds them with ctypes, see
 * INTEGRATION.md). Conventions:
 *   - all pointers are DEVICE pointers (fp32 row-major, uint8 flags, int64
 *     indices) unless marked "host"; memory is owned by the caller (PyTorch's
 *     caching allocator), the library never allocates on the hot path;
 *   - every call is asynchronous on `stream` (a hipStream_t passed as void*);
 *   - return 0 on success, DRPO_EINVAL / DRPO_EHIP / DRPO_EUNSUPPORTED
 *     otherwise, with a message in drpo_last_error() (thread-local);
 *   - noise: a non-NULL eps pointer is "parity mode" (the caller supplies the
 *     reference's standard-normal draws); NULL means Philox4x32-10 on the device
 *     keyed by (seed, ctr, call-site).
 * Reference citations are path:line in the reference repository.
 */
#ifndef DRPO_HIP_H
#define DRPO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* drpo_stream_t; /* hipStream_t */

enum { DRPO_OK = 0, DRPO_EINVAL = 1, DRPO_EHIP = 2, DRPO_EUNSUPPORTED = 3 };

/* activation ids used by the MLP descriptors (src/torch_util.py:169-178) */
enum { DRPO_ACT_NONE = 0, DRPO_ACT_RELU = 1, DRPO_ACT_SILU = 2, DRPO_ACT_TANH = 3 };

/* device environment ids for the batched constraint functions (src/smbpo.py:63-65) */
enum { DRPO_ENV_POINT_ROBOT = 0, DRPO_ENV_QUADROTOR = 1, DRPO_ENV_CARTPOLE = 2, DRPO_ENV_TRACKING = 3 };

/* ---------------------------------------------------------------- library */
int drpo_version(void);
int64_t drpo_abi_sizeof(const char* struct_name);   /* binding self-check */
const char* drpo_last_error(void);
/* SHA-256 (hex) of the csrc/include sources this binary was built from; the Python
 * binding refuses a library whose digest differs from the sources beside it */
const char* drpo_build_digest(void);
int drpo_event_create(void** ev);
int drpo_event_destroy(void* ev);
int drpo_event_record(void* ev, drpo_stream_t stream);
int drpo_event_elapsed_ms(float* ms /* host */, void* start, void* stop);
int drpo_stream_wait_event(drpo_stream_t stream, void* ev);   /* hipStreamWaitEvent (cross-stream hand-off) */

/* ---------------------------------------------------------------- rollout
 * Replaces SMBPO.rollout (src/smbpo.py:229-249) together with
 * BatchedGaussianEnsemble.sample (src/dynamics.py:198-203, _forward1 :112-122),
 * SquashedGaussianPolicy.act(eval=False) (src/policy.py:77-97), the env
 * check_done / check_violation / get_constraint_values round trips
 * (src/smbpo.py:63-65) and ConstraintSafetySampleBuffer.extend into the virtual
 * buffer (src/sampling.py:128-145). Rows that are done leave the batch; the
 * buffer receives each step's surviving rows in order, as the reference's
 * next_states[~dones] compaction does. Engine 1 runs one kernel per horizon
 * step; engine 2 (default) keeps each row tile on one workgroup for the whole
 * horizon and orders the rows into the buffer afterwards.                   */
typedef struct {
  int S, A, C, Ha, Hm, B, H;
  int env_id, tracking_surr_start, tracking_n_surr;
  double env_thr0, env_thr1;     /* quadrotor: x/z_threshold (safe-control-gym); cartpole: x_threshold,
                                    th_threshold (SafeInvertedPendulumEnv); unused otherwise */
  const float *aW1, *ab1, *aW2, *ab2, *aW3, *ab3;          /* actor: packed weight mirrors + biases */
  const float *mW1, *mb1, *mW2, *mb2, *dW1, *db1, *dW2, *db2, *lW1, *lb1, *lW2, *lb2; /* ensemble: packed mirrors [E] (member stride drpo_packed_size) + biases [E][out] */
  const float *norm_mean, *norm_std, *min_lv, *max_lv;
  const int* members;            /* host [H]: elite member per step (random.choice, src/dynamics.py:199) */
  const float* replay_states;    /* real buffer states, physical layout */
  int64_t replay_ptr, replay_cap;
  const int64_t* init_idx;       /* [B] chronological indices (np.random.choice) or NULL: device sampling w/o replacement */
  const float* eps_a;            /* [H][B][A] or NULL */
  const float* eps_m;            /* [H][B][S+1] or NULL */
  uint64_t seed, ctr;
  float *vs, *va, *vs2, *vr, *vh;  /* virtual buffer components */
  uint8_t *vd, *vv;
  int64_t* vptr;                 /* device int64 write pointer, advanced by the rollout */
  int64_t vcap;
  void* workspace;               /* drpo_rollout_workspace_size bytes; one rollout at a time per workspace */
  int rows_per_tile;             /* 16 or 32, 0 = auto */
  void** step_events;            /* optional [2*H] events: engine 1 records pair t around step t's kernel,
                                    engine 2 records pair 0 around the fused horizon kernel */
  int engine;                    /* 0 auto, 1 one launch per horizon step, 2 fused horizon (persistent per tile) */
  int eps_layout;                /* eps_a/eps_m rows: 0 compacted per step (reference draw order; engine 1),
                                    1 original batch row (row i of step t = trajectory i; engine 2) */
} drpo_rollout_desc_t;

size_t drpo_rollout_workspace_size(int B, int S, int H);
size_t drpo_rollout_count_offset(int B, int S, int H); /* byte offset of the int64 row count in the workspace */
int drpo_rollout(const drpo_rollout_desc_t* d /* host */, drpo_stream_t stream);

/* batched env constraint functions, e.g. PointRobot.get_constraint_values /
 * check_violation / check_done (src/env/point_robot.py:96-131); h is [n][C] */
int drpo_env_constraints(int env_id, int tracking_surr_start, int tracking_n_surr, double env_thr0,
                         double env_thr1, const float* states, int64_t n, int S, uint8_t* done,
                         uint8_t* violation, float* h, drpo_stream_t stream);

/* ---------------------------------------------------------------- safety shields
 * Real-env step shield (SMBPO.step_generator, src/smbpo.py:127-136) and the
 * evaluation shields of sample_episodes_batched (src/sampling.py:423-439).
 * drpo_shield_mix writes the linear shield's K candidate actions
 * mix_i = a_safe*(K-1-i)/(K-1) + a_perf*(1-(K-1-i)/(K-1)) as [K][n][A] (scored by one
 * constraint-critic forward over K*n rows); drpo_shield_select picks per row:
 * mode 0 a_perf; mode 1 a_safe where max_C q > threshold (q [n][C]); mode 2 linear
 * shield: a_safe, overridden by mix_i wherever max_C q_i <= threshold (q [K][n][C]). */
int drpo_shield_mix(const float* a_perf, const float* a_safe, int64_t n, int A, int K, float* mixes,
                    drpo_stream_t stream);
int drpo_shield_select(const float* q, int K, int64_t n, int C, int A, int mode, float threshold, const float* a_perf,
                       const float* a_safe, const float* mixes, float* out, drpo_stream_t stream);

/* B distinct indices in [0, N): production stand-in for random_choice(replace=False)
 * (src/torch_util.py:41-48) */
int drpo_sample_without_replacement(int64_t* out, int64_t B, int64_t N, uint64_t seed, uint64_t ctr,
                                    drpo_stream_t stream);

/* ---------------------------------------------------------------- MLPs
 * Fused forward / backward-data / weight-gradient passes for mlp() nets
 * (src/torch_util.py:190-211) and BatchedLinear ensembles (src/dynamics.py:26-52,
 * nbatch = ensemble members). Used by the SAC update (src/ssac.py:437-578),
 * the ensemble fit (src/dynamics.py:143-187) and every network forward.      */
typedef struct {
  const float* W; /* packed forward mirror of the [dout][din] weight (drpo_pack_weights) */
  const float* b; /* [dout] */
  int din, dout, act;
  float* sy;      /* optional: post-activation save [rows][dout] */
  float* sz;      /* optional: pre-activation save */
  int64_t wstride, bstride; /* per batch item (ensemble member): packed-mirror / bias strides */
} drpo_mlp_layer_t;

typedef struct {
  int nl;
  drpo_mlp_layer_t L[3];
} drpo_mlp_net_t;

/* squashed-Gaussian policy head fused into a forward pass: applied to net[0]'s
 * final output (2A columns = [mu | log-std pre-activation]), src/policy.py:88-97 */
typedef struct {
  int mode;            /* 0 none, 1 sample (Normal.sample), 2 rsample, 3 mean only (tanh(mu)) */
  int A;
  const float* eps;    /* [rows][A] recorded draws, or NULL: Philox (launch seed/ctr, this site) */
  uint32_t site;
  float *a, *logp, *u, *e, *amean;   /* optional outputs */
} drpo_policy_head_t;

typedef struct {
  const float* src[3]; /* column-concatenated input sources (e.g. torch.cat([s, a], -1)) */
  int cols[3];
  int ld[3];
  int64_t sstride[3];
  const float* nmean;  /* optional (src[0] - mean) / (std + 1e-6) (src/normalization.py:22-23) */
  const float* nstd;
  float* save_x;       /* optional save of the assembled input */
  drpo_mlp_net_t net[3];
  int nnets;
  int trunk;           /* 1: net[0] trunk, net[1..] heads on its output */
  int64_t rows;
  int nbatch;
  drpo_policy_head_t head;   /* multi-job launches only (mode 0 elsewhere) */
  int split_heads;     /* trunk mode, single launches: one workgroup per (row tile, head); each
                          recomputes the trunk (only head 1's workgroup saves it) -- twice the
                          workgroups for small ensembles (fit: 16 tiles x 7 members) */
  float* ccb_out;      /* multi-job launches, trunk job with paired heads (the constraint critic,
                          src/ssac.py:46-92): per-row max over the C constraints of the quantile
                          bound mu + ccb_ratio * std(log-std raw) (ccb_dist) or of mu, formed from
                          the heads' outputs in the launch (drpo_cc_head's arithmetic,
                          src/ssac.py:474-494,536-560); NULL: none */
  int ccb_dist;
  float ccb_ratio, ccb_lmin, ccb_lmax;
  /* multi-job launches: */
  int pair;            /* non-trunk job, 2 nets of ONE shape on the same input (the twin critics; the
                          actor and the safe actor): ONE workgroup runs both as paired layers (one
                          staging, one k-loop per layer pair) instead of one workgroup per net */
  drpo_policy_head_t head2;   /* pair jobs: the fused head of net[1] (head: net[0]'s) */
  drpo_mlp_net_t pre;  /* chain (pre.nl > 0): a policy net run first, in the same workgroup, on the
                          src[0] columns; its head (pre_head, mode 1 or 2) samples the action that
                          is this job's src[1] column block (cols[1] == A) straight from LDS: the
                          next-state policy feeding the target critics / certificate
                          (src/ssac.py:284-294,387-400) without a launch or an HBM round trip */
  drpo_policy_head_t pre_head;
  drpo_mlp_net_t post; /* post chain (post.nl > 0; a trunk job with ccb_out): a net run after the bound in
                          the same workgroup on [src[0] columns (cols[0] wide), the bound] -- the
                          MLPMultiplier lam(s, max_C Qc_ub(s, a)) of src/ssac.py:473-478,548-552
                          without its own launch; its layer saves as any net's */
  float* post_x;       /* optional save of the post net's assembled input [rows][cols[0] + 1] */
} drpo_mlp_fwd_t;

typedef struct {
  const float* W;      /* packed TRANSPOSED mirror of the [dout][din] weight */
  int din, dout, act;
  const float* sy;
  const float* sz;
  float* dz;           /* optional save of dL/dZ for weight gradients */
  int64_t wstride;
  float* dz2;          /* split_heads trunk layers: the second head's partial dL/dZ (trunk
                          dZ = dz + dz2) */
} drpo_mlp_bwd_layer_t;

typedef struct {
  int nl;
  drpo_mlp_bwd_layer_t L[3];
  const float* gout;   /* dL/d(output) [rows][dout_last] */
  float* dx;           /* optional dL/d(input) for input columns [dx_col0, dx_col0 + dx_cols) */
  int dx_col0, dx_cols, dx_accumulate;
} drpo_mlp_bwd_net_t;

typedef struct {
  drpo_mlp_bwd_net_t net[3];
  int nnets;
  int trunk;
  int64_t rows;
  int nbatch;
  int split_heads;     /* trunk mode, single launches, trunk dx unused: one workgroup per (row
                          tile, head) backs its head's gradient through the trunk (linear in
                          the head gradients), writing dz (head 1) / dz2 (head 2) */
  int upstream;        /* where the output gradients come from: DRPO_UPSTREAM_* */
} drpo_mlp_bwd_t;

/* The model fit's NLL loss (drpo_ens_loss's arithmetic, src/dynamics.py:136-153,236-253)
 * as the upstream of the ensemble backward launch (drpo_mlp_backward_ens): the head
 * outputs' gradients are formed in-kernel and the loss partials are left for the
 * deferred reduction (drpo_mlp_wgrad_reduce). */
typedef struct {
  const float *D, *LVR;        /* diff / raw log-var head outputs [Z][b][S+1] */
  const float* s;              /* raw states [Z][b][S] (member stride s_zstride) */
  int64_t s_zstride;
  const float* t;              /* targets [Z][b][S+1] */
  int64_t t_zstride;
  int64_t b;                   /* rows per member */
  int S, Z;
  const float *minlv, *maxlv;
  const float* gscale;         /* optional device scale of the gradients (NULL = 1) */
  float* part;                 /* loss workspace (drpo_ens_loss_workspace_size) */
} drpo_ens_upstream_t;

/* The actor update's output gradients (src/ssac.py:458-527), formed in-kernel by its
 * backward launches (drpo_mlp_backward_multi_actor): what drpo_actor_upstream and
 * drpo_squash_backward compute as separate launches. */
typedef struct {
  int64_t B;
  int C, A, distributional;
  float std_ratio, log_std_min, log_std_max;
  const float* lams;            /* MLPMultiplier pre-transform outputs [B], or NULL: fixed_lam */
  float lam_upper_bound, fixed_lam, clamp_lb, clamp_ub;
  const float* u[2];            /* pre-tanh samples of the actor [0] / safe actor [1] [B][A] */
  const float* e[2];            /* their standard-normal draws [B][A] */
  const float* dA[2];           /* dL/d action [B][A] */
  const float* dA2[2];          /* optional second term of dL/d action (NULL) */
  const float* logp;            /* actor log-probs [B] */
  const float* log_alpha;       /* the actor's log-prob terms scaled by exp(*log_alpha) * lp_scale; NULL: none */
  float lp_scale, target_entropy;
  float* alpha_sum;             /* per row tile: sum(logp + target_entropy) of the actor's rows, or NULL
                                   (one float per 16-row tile, overwritten; drpo_optim_seg_t.grad_sum_n) */
} drpo_actor_head_t;

/* drpo_mlp_bwd_t.upstream */
#define DRPO_UPSTREAM_GOUT 0     /* the nets' gout arrays */
#define DRPO_UPSTREAM_CRITIC 1   /* twin-critic job: net k's output gradient is (q_k - y) / B with the soft
                                    Bellman target y of the launch's critic head; adds the critic loss */
#define DRPO_UPSTREAM_CERT 2     /* constraint-critic job (trunk + mean [+ log-std] heads): the
                                    certificate loss gradients of the launch's critic head; adds its loss */
#define DRPO_UPSTREAM_ENS 3      /* ensemble job (trunk + diff / log-var heads): the NLL gradients of the
                                    launch's drpo_ens_upstream_t; writes its loss partials */
#define DRPO_UPSTREAM_ACTOR_CC 4 /* constraint critic at (s, a): lam / B on the max-C certificate bound of
                                    the launch's drpo_actor_head_t (src/ssac.py:474-488) */
#define DRPO_UPSTREAM_SAFE_CC 5  /* constraint critic at (s, a_safe): 1 / B on its max-C bound (:490-494) */
#define DRPO_UPSTREAM_NEG_MEAN 6 /* single net with one output: -1 / B (the actor loss's -mean(Q_k)) */
#define DRPO_UPSTREAM_SQUASH 7   /* actor (net 0 of the launch's head: [0]) / safe actor ([1]): the
                                    squashed-Gaussian backward of the head's action gradients */
#define DRPO_UPSTREAM_SQUASH_SAFE 8

typedef struct {
  const float* dz; /* [rows][dout] */
  const float* y;  /* layer input [rows][din] */
  float* gW;       /* gW += dZ^T Y (no two items of one launch may share gW) */
  float* gb;       /* gb += colsum(dZ) */
  int dout, din;
  int64_t rows;
  int64_t zstride, ystride, gwstride, gbstride;
  int nbatch;
  float* sq;       /* optional clip partials: sq[sq_off + t] = sum of squares of the
                      FINISHED gradient (weights + bias) of output tile t of this item,
                      t < drpo_mlp_wgrad_tiles(item) (summed by drpo_optim_step) */
  int sq_off;
  const float* dz2;  /* optional second dL/dZ term, same layout as dz: the product is
                        (dz + dz2)^T y (a split-heads backward leaves the trunk's dZ as
                        the sum of the two heads' shares) */
} drpo_wgrad_item_t;

/* the reduction step of drpo_ens_loss, as data: run by drpo_mlp_wgrad_reduce */
typedef struct {
  const float* part;   /* the loss workspace */
  int nbx, Z, S1;
  const float *minlv, *maxlv;
  float weight;
  const float* gscale;
  float *mse, *loss, *gmin, *gmax;
} drpo_ens_reduce_t;

/* the safe-SAC critic losses of one update_critic (src/ssac.py:284-435): drpo_critic_head
 * (csrc/sac.hip) or fused into drpo_mlp_backward_multi_head */
typedef struct {
  int64_t B;
  int C;
  int distributional, deterministic_backup;
  float discount, qc_td_bound, lmin, lmax;
  const float* log_alpha;
  const float *r, *h;
  const uint8_t* d;
  const uint8_t* dc;    /* certificate-target done flags (robust branch: model-predicted); NULL = d */
  const float *q0t, *q1t, *logp2;
  const float *mu_t, *ls_t;
  const float* eps3;
  uint64_t seed, ctr;
  const float *q0, *q1;
  const float *mu, *ls;
  float *dq0, *dq1, *dmu, *dls;
  float* loss; /* [2] accumulated: critic loss, constraint-critic loss */
  float* loss_part;   /* drpo_mlp_backward_multi_head only: per-workgroup loss partials instead of
                         atomics into loss: [3][row tiles] = twin 0, twin 1, certificate (summed by
                         a drpo_mlp_wgrad_sums reduction) */
  /* constrained_fcn='cost' (src/ssac.py:306-310): certificate target = violation + discount *
     (1 - done) * mu_t, MSE loss (distributional must be 0); v = the batch's violation flags */
  int cost;
  const uint8_t* v;
} drpo_critic_head_t;

int drpo_mlp_forward(const drpo_mlp_fwd_t* desc /* host */, drpo_stream_t stream);
/* Up to 8 independent forward jobs (different inputs / nets, e.g. every forward of
 * one SAC loss that does not depend on another) in ONE launch, each with an
 * optional fused policy head. jobs_dev: the same descriptors in device memory
 * (read by the kernel; static across calls), jobs_host: for the grid. */
int drpo_mlp_forward_multi(const drpo_mlp_fwd_t* jobs_host, const drpo_mlp_fwd_t* jobs_dev, int njobs, uint64_t seed,
                           uint64_t ctr, drpo_stream_t stream);
int drpo_mlp_backward(const drpo_mlp_bwd_t* desc /* host */, drpo_stream_t stream);
/* independent backward-data jobs in one launch (descriptors in device memory) */
int drpo_mlp_backward_multi(const drpo_mlp_bwd_t* jobs_host, const drpo_mlp_bwd_t* jobs_dev, int njobs,
                            drpo_stream_t stream);
/* the same with the critic losses fused in (update_critic, src/ssac.py:284-456): jobs with
 * upstream = DRPO_UPSTREAM_CRITIC / _CERT form their output gradients from `head` (the
 * forward outputs, targets and batch of drpo_critic_head_t; its dq0 / dq1 / dmu / dls are
 * not written, loss[0] / loss[1] are accumulated) -- no separate head launch */
int drpo_mlp_backward_multi_head(const drpo_mlp_bwd_t* jobs_host, const drpo_mlp_bwd_t* jobs_dev, int njobs,
                                 const drpo_critic_head_t* head /* host */, drpo_stream_t stream);
/* the actor update's backward launches with actor_upstream / squash_backward fused in */
int drpo_mlp_backward_multi_actor(const drpo_mlp_bwd_t* jobs_host, const drpo_mlp_bwd_t* jobs_dev, int njobs,
                                  const drpo_actor_head_t* head /* host */, drpo_stream_t stream);
/* the model fit's backward with the NLL loss fused in: desc->upstream = DRPO_UPSTREAM_ENS,
 * trunk + paired diff / log-var heads. reduce_out receives the deferred reduction
 * (mse / loss / gmin / gmax / weight: from `red_in`, partial layout from this launch). */
int drpo_mlp_backward_ens(const drpo_mlp_bwd_t* desc /* host */, const drpo_ens_upstream_t* up /* host */,
                          const drpo_ens_reduce_t* red_in /* host */, drpo_ens_reduce_t* reduce_out,
                          drpo_stream_t stream);
/* The model fit step's forward + NLL + backward-data in ONE launch (csrc/fit.hip;
 * BatchedGaussianEnsemble.fit's compute_loss + loss.backward(), src/dynamics.py:112-122,
 * 136-153,236-253): replaces drpo_mlp_forward(fwd) + drpo_mlp_backward_ens(bwd, up) for
 * the ensemble trunk [S+A <= 64 -> H -> H] with diff / log-var heads [H -> H -> S+1 <= 16]
 * (swish hidden layers, H = 200 | 256). fwd: the split-heads forward descriptor with its
 * y saves (head output saves and z saves are not written); bwd: the split-heads backward
 * descriptor (trunk dz + dz2); up: as for drpo_mlp_backward_ens (D / LVR unused). Writes
 * the same saves, dZ and loss partials as the two launches. */
int drpo_ens_fit_fb(const drpo_mlp_fwd_t* fwd /* host */, const drpo_mlp_bwd_t* bwd /* host */,
                    const drpo_ens_upstream_t* up /* host */, const drpo_ens_reduce_t* red_in /* host */,
                    drpo_ens_reduce_t* reduce_out, drpo_stream_t stream);
/* Weight gradients of up to 16 layers (items) in ONE launch: gW += dZ^T Y, gb +=
 * colsum(dZ) (the autograd of nn.Linear / BatchedLinear, src/dynamics.py:26-52,
 * src/torch_util.py:190-211), split into (output tile x row chunk) workgroups whose
 * partial tiles are combined in a fixed order by the tile's last workgroup (no float
 * atomics: deterministic). workspace: drpo_mlp_wgrad_workspace_size(items, n) bytes,
 * ZEROED by the caller once before its first use (the launch leaves it zeroed). */
size_t drpo_mlp_wgrad_workspace_size(const drpo_wgrad_item_t* items /* host */, int n);
/* output tiles of one item (the number of sq partials it writes) */
int drpo_mlp_wgrad_tiles(const drpo_wgrad_item_t* item /* host */);
int drpo_mlp_wgrad(const drpo_wgrad_item_t* items /* host */, int n, void* workspace, size_t workspace_bytes,
                   drpo_stream_t stream);
/* drpo_mlp_wgrad plus one extra workgroup running a deferred ensemble-loss
 * reduction (drpo_ens_loss_partials); red may be NULL */
int drpo_mlp_wgrad_reduce(const drpo_wgrad_item_t* items /* host */, int n, const drpo_ens_reduce_t* red /* host */,
                          void* workspace, size_t workspace_bytes, drpo_stream_t stream);
/* drpo_mlp_wgrad plus one extra workgroup adding up partial sums in a fixed order:
 * *out = part[0] + part[1] + ... + part[n-1] for each of nsums (<= 4) entries (the
 * per-workgroup loss partials of drpo_mlp_backward_multi_head; no float atomics) */
typedef struct {
  const float* part;
  int n;
  float* out;
} drpo_sum_t;
int drpo_mlp_wgrad_sums(const drpo_wgrad_item_t* items /* host */, int n, const drpo_sum_t* sums /* host */,
                        int nsums, void* workspace, size_t workspace_bytes, drpo_stream_t stream);

/* The Adam step fused into the weight-gradient launch (no clip, no data-parallel
 * exchange between the gradient and the step: the single-process model fit,
 * src/dynamics.py:155-183 with torch.optim.Adam): the workgroup that finishes an output
 * tile applies Adam to it (the drpo_optim_step arithmetic, so results are bitwise
 * those of drpo_mlp_wgrad + drpo_optim_step) and refreshes the tile's packed mirrors;
 * the optional reduction block does the same for the log-var bounds. The gradient
 * buffer is consumed without being written (it must hold zeros or terms to add; any
 * nonzero term is cleared, like drpo_optim_step's zero_grad). */
struct drpo_pack_map_s;
typedef struct {
  const float* g;             /* base of the flat gradient the items' gW / gb (and gmin / gmax) point into */
  float *p, *m, *v;           /* the group's data and Adam moments, indexed like g */
  float lr_over_bc1, bc2_sqrt, beta1, beta2, eps, weight_decay;
  const struct drpo_pack_map_s* map;      /* device pack map of the group (mirrors refreshed) or NULL */
  const struct drpo_pack_map_s* map_host; /* its host copy (which matrix each item is) */
} drpo_wgrad_adam_t;
int drpo_mlp_wgrad_adam(const drpo_wgrad_item_t* items /* host */, int n, const drpo_ens_reduce_t* red /* host or NULL */,
                        const drpo_wgrad_adam_t* adam /* host */, void* workspace, size_t workspace_bytes,
                        drpo_stream_t stream);

/* ---------------------------------------------------------------- packed weight mirrors
 * Every MLP kernel streams weights from fragment-linear mirrors of the PyTorch
 * [nbatch][dout][din] tensors (layout: csrc/pack.hip). The mirrors are refreshed
 * by one drpo_pack_weights launch per parameter group after it changes.        */
typedef struct {
  const float* W;     /* [nbatch][dout][din], member stride wstride */
  float* P;           /* forward mirror (or NULL), member stride pstride */
  float* PT;          /* transposed (backward-data) mirror (or NULL), stride ptstride */
  int din, dout, nbatch;
  int64_t wstride, pstride, ptstride;
} drpo_pack_item_t;

int64_t drpo_packed_size(int din, int dout); /* floats per mirror of one [dout][din] matrix */
int drpo_pack_weights(const drpo_pack_item_t* items /* host, <= 16 */, int n, drpo_stream_t stream);

/* ---------------------------------------------------------------- SAC heads
 * (src/ssac.py:284-578, src/smbpo.py:251-279, src/policy.py:89-97)            */
typedef struct {
  const float *s, *a, *s2, *r, *h;
  const uint8_t *d, *v;
  int64_t len;          /* rows available, or -1: min(*ptr_dev, cap) read on the device */
  const int64_t* ptr_dev;
  int64_t cap;
} drpo_buffer_view_t;

/* mixed real/virtual minibatch (src/smbpo.py:253-270; SampleBuffer.sample src/sampling.py:147-151) */
int drpo_sample_batch(const drpo_buffer_view_t* real, const drpo_buffer_view_t* virt, int n_real, int B, int S, int A,
                      int C, const int64_t* idx_real, const int64_t* idx_virt, uint64_t seed, uint64_t ctr,
                      float reward_scale, float alive_bonus, float constraint_scale, float constraint_offset, float* s,
                      float* a, float* s2, float* r, uint8_t* d, uint8_t* v, float* h, drpo_stream_t stream);

/* squashed Gaussian (src/policy.py:89-97, src/squashed_gaussian.py): mode 0 sample,
 * 1 rsample, 2 mean (tanh(mu)), 3 distribution parameters (loc -> u, scale -> e); raw = [mu | log-std pre-activation] [B][2A] */
int drpo_policy_head(const float* raw, int64_t B, int A, int mode, const float* eps, uint64_t seed, uint64_t ctr,
                     uint32_t site, float* a, float* logp, float* u, float* e, float* amean, drpo_stream_t stream);

/* ConstraintCritic.forward per-constraint outputs (src/ssac.py:75-92): mode 0 uncertainty
 * q = mu + std_ratio*std, mode 1 sample (std, mu + clamp(eps, +-2)*std); eps NULL -> Philox */
int drpo_cc_dist(const float* mu, const float* lsraw, int64_t n, int mode, float std_ratio, float log_std_min,
                 float log_std_max, const float* eps, uint64_t seed, uint64_t ctr, float* std_out, float* q,
                 drpo_stream_t stream);

/* ConstraintCritic log-std clamp + quantile bound mu + std_ratio*std, max over C
 * (src/ssac.py:64-92, _get_qc :588-600) */
int drpo_cc_head(const float* mu, const float* lsraw, int64_t B, int C, int distributional, float std_ratio,
                 float log_std_min, float log_std_max, float* ubmax, int* argmax, drpo_stream_t stream);


/* compute_target + compute_cons_target + critic / constraint-critic losses and
 * their output gradients (src/ssac.py:284-435) */
int drpo_critic_head(const drpo_critic_head_t* p /* host */, drpo_stream_t stream);

/* dL/d outputs of the critic and constraint critic for actor_loss (src/ssac.py:458-505) */
int drpo_actor_upstream(int64_t B, int C, int distributional, float std_ratio, float log_std_min, float log_std_max,
                        const float* lams, const float* mu_a, const float* ls_a, const float* mu_s, const float* ls_s,
                        float* gq, float* gmu_a, float* gls_a, float* gmu_s, float* gls_s,
                        float lam_upper_bound /* > 0: lams holds the MLPMultiplier's raw output x and
                                                 lam = ub/2 (1 + tanh(2x/ub)) (src/ssac.py:107-111) is
                                                 applied here; 0: lams holds lam */,
                        float fixed_lam, float clamp_lb, float clamp_ub /* lams == NULL (scalar-multiplier
                                                 solver, mlp_multiplier = False): lam = fixed_lam and the
                                                 certificate term is clamp(Qc, lb, ub) (src/ssac.py:481-484) */,
                        drpo_stream_t stream);

/* chain rule through rsample/tanh/log_prob to the actor head; alpha-loss sum */
int drpo_squash_backward(int64_t B, int A, const float* raw, const float* u, const float* e, const float* dA,
                         const float* dA2 /* optional second dL/da term, summed: dA + dA2 */, const float* log_alpha, float lp_scale, const float* logp, float target_entropy,
                         float* alpha_sum, float* draw, drpo_stream_t stream);

/* d alpha_loss / d log_alpha (src/ssac.py:498-501) */
int drpo_alpha_grad(const float* log_alpha, const float* alpha_sum, int64_t B, float* grad, drpo_stream_t stream);

/* multiplier loss gradient w.r.t. the MLPMultiplier output (src/ssac.py:529-568). x == NULL
 * (scalar multiplier, src/ssac.py:564-566): *loss accumulates sum_i clamp(actor_qc_i -
 * threshold, lb, ub), the penalty sum of -mean(softplus(m) * penalty); gx unused. */
int drpo_multiplier_head(int64_t B, const float* x, const float* safe_qc, const float* actor_qc, float threshold,
                         float penalty_lb, float penalty_ub, float upper_bound, float lam_epsilon, float* gx,
                         float* loss, drpo_stream_t stream);
/* MLPMultiplier.forward output transform (src/ssac.py:107-111) */
int drpo_multiplier_out(int64_t B, const float* x, float upper_bound, float* lam, drpo_stream_t stream);

/* ---------------------------------------------------------------- dynamics ensemble
 * BatchedGaussianEnsemble (src/dynamics.py:112-253); the MLP passes use
 * drpo_mlp_forward/backward/wgrad with nbatch = ensemble members.              */
/* fit / holdout minibatch gather by chronological replay index (src/dynamics.py:156-166,
 * 175-177); idx NULL -> Philox randint(n) with (seed, ctr); ptr_dev overrides ptr */
int drpo_ens_gather(const float* states, const float* actions, const float* next_states, const float* rewards,
                    int64_t ptr, const int64_t* ptr_dev, int64_t cap, int64_t rows, const int64_t* idx, uint64_t seed,
                    uint64_t ctr, int S, int A, float* xs, float* xa, float* xt, drpo_stream_t stream);
/* the minibatches of `steps` consecutive fit steps in one launch: step k fills rows
 * [k*rows, (k+1)*rows) of xs / xa / xt from idx[k*rows ..] (or Philox counter ctr + k) */
int drpo_ens_gather_steps(const float* states, const float* actions, const float* next_states, const float* rewards,
                          int64_t ptr, const int64_t* ptr_dev, int64_t cap, int64_t rows, int64_t steps,
                          const int64_t* idx, uint64_t seed, uint64_t ctr, int S, int A, float* xs, float* xa,
                          float* xt, drpo_stream_t stream);
/* mu = diff + [s, 0], soft log-var clamp, optional sample -> (s', r)
 * (_forward1 / _forward_all / sample / elite_samples, src/dynamics.py:112-134,198-234) */
int drpo_ens_head(const float* D, const float* LVR, const float* s, int64_t s_zstride, int64_t n, int S, int nz_out,
                  const float* minlv, const float* maxlv, const int* zsel, const float* eps, uint64_t seed,
                  uint64_t ctr, float* mu, float* lv, float* s2, float* r, drpo_stream_t stream);
/* per-member NLL (_mse_loss, src/dynamics.py:236-253), total compute_loss (:143-153)
 * and, when gD != NULL, its gradients (scaled by *gscale if given; gmin/gmax are
 * accumulated into). Row blocks leave partial sums in the workspace
 * (drpo_ens_loss_workspace_size(b, S, Z) bytes; one call at a time per workspace),
 * reduced in a fixed order by a one-block launch. */
size_t drpo_ens_loss_workspace_size(int64_t b, int S, int Z);
int drpo_ens_loss(const float* D, const float* LVR, const float* s, int64_t s_zstride, const float* t,
                  int64_t t_zstride, int64_t b, int S, int Z, const float* minlv, const float* maxlv, float weight,
                  const float* gscale, float* mse, float* loss, float* gD, float* gLVR, float* gmin, float* gmax,
                  void* workspace, drpo_stream_t stream);
/* drpo_ens_loss without its reduction launch: the reduction is described in
 * *reduce_out and runs as the extra last workgroup of the next
 * drpo_mlp_wgrad_reduce (the fit step's weight-gradient launch, which the
 * reduction does not depend on) -- one launch fewer per fit step. */
int drpo_ens_loss_partials(const float* D, const float* LVR, const float* s, int64_t s_zstride, const float* t,
                           int64_t t_zstride, int64_t b, int S, int Z, const float* minlv, const float* maxlv,
                           float weight, const float* gscale, float* mse, float* loss, float* gD, float* gLVR,
                           float* gmin, float* gmax, void* workspace, drpo_ens_reduce_t* reduce_out,
                           drpo_stream_t stream);
/* The deferred reduction of drpo_ens_loss_partials / drpo_mlp_backward_ens as its own
 * one-block launch (replaces the reduction step of BatchedGaussianEnsemble.fit,
 * src/dynamics.py:143-153,163-171): per-member NLL, the step loss and the log-var
 * bound gradients ACCUMULATED into gmin / gmax (no optimizer step). The member-
 * sharded fit runs it on a side stream so the bounds' all-reduce overlaps the
 * members' fused weight-gradient + Adam launch. */
int drpo_ens_loss_reduce(const drpo_ens_reduce_t* red /* host */, drpo_stream_t stream);

/* ---------------------------------------------------------------- optimizer
 * torch.optim.Adam (coupled L2), clip_grad_norm_, update_ema (src/ssac.py:446-455,
 * src/torch_util.py:223-226), over flat parameter groups                       */
int drpo_grad_sumsq_blocks(int64_t n);
int drpo_grad_sumsq(const float* g, int64_t n, float* partial, drpo_stream_t stream);
int drpo_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr_over_bc1, float bc2_sqrt, float beta1,
              float beta2, float eps, float weight_decay, const float* clip_partial, int n_partial, float max_norm,
              const float* lr_scale, drpo_stream_t stream);
int drpo_ema(float* target, const float* source, int64_t n, float rate, drpo_stream_t stream);

/* Fused optimizer step over segments of flat groups: clip coefficient from the
 * partial sums (clip_grad_norm_, src/ssac.py:450-451), Adam (src/defaults.py:4),
 * gradient zeroing, EMA of a target group (src/torch_util.py:223-226) and the
 * packed-mirror refresh, in ONE launch.                                        */
typedef struct drpo_pack_map_s { /* device memory: where each weight matrix of a group lives */
  int nlayers;
  int64_t off[16];            /* flat offset of the [nbatch][dout][din] weight */
  int din[16], dout[16], nbatch[16];
  int64_t poff[16];           /* offset of its packed mirrors (forward / transposed / target) */
  float *P, *PT, *Pt;         /* mirrors (PT, Pt may be NULL) */
} drpo_pack_map_t;

typedef struct {
  float *p, *g, *m, *v;       /* flat group (element indices are absolute) */
  int64_t start, end;
  int adam;                   /* 0: no Adam update (EMA / pack only) */
  const float* partial;       /* clip partial sums (drpo_grad_sumsq[_multi]) or NULL */
  int n_partial;
  float max_norm;
  float lr_over_bc1, bc2_sqrt, beta1, beta2, eps, weight_decay;
  int zero_grad;              /* write g = 0 after use */
  float* ema_target;          /* optional: target = rate*p + keep*target */
  float ema_rate, ema_keep;
  const drpo_pack_map_t* map; /* optional (device): packed mirrors to refresh */
  const float* grad_from_sum; /* optional (device scalar): the gradient of element i is
                                 -exp(p_i) * (*grad_from_sum / grad_sum_rows) instead of g[i]:
                                 d alpha_loss / d log_alpha from the alpha-loss sum of
                                 drpo_squash_backward (src/ssac.py:498-501), so the SAC
                                 temperature needs no separate gradient launch */
  int64_t grad_sum_rows;
  int grad_from_sum_kind;     /* 0: -exp(p_i) * sum / rows (the SAC temperature, alpha loss);
                                 1: -sigmoid(p_i) * sum / rows (the scalar Lagrange multiplier,
                                    -mean(softplus(m) * penalty), src/ssac.py:564-566);
                                 2: -sum / rows (use_log_alpha_loss, src/ssac.py:499) */
  float grad_scale;           /* gradient multiplier applied before clip and Adam (the clip
                                 norm is that of the scaled gradient): 1/G folds the data-
                                 parallel mean into the step after a SUM all-reduce. 0 is
                                 read as 1, so zero-initialised descriptors keep plain grads */
  int grad_sum_n;             /* grad_from_sum holds this many partial sums, added in order (0 = 1) */
  const drpo_pack_map_t* map_host; /* optional host copy of *map: the launch then covers each
                                 weight matrix in 4x4 blocks (16-byte loads / stores per row,
                                 16-byte mirror stores per row and per column) instead of
                                 runs of 4 flat elements with scattered transposed-mirror
                                 stores */
} drpo_optim_seg_t;

int drpo_optim_step(const drpo_optim_seg_t* segs /* host, <= 8 */, int n, drpo_stream_t stream);
int drpo_grad_sumsq_multi(const float* const* g /* host arrays */, const int64_t* n, float* const* partial_out, int cnt,
                          drpo_stream_t stream);

/* Normalizer.fit / forward (src/normalization.py:14-23) */
size_t drpo_normalizer_workspace_size(int64_t N, int S);
int drpo_normalizer_fit(const float* X, int64_t N, int S, float* mean, float* std, void* workspace,
                        drpo_stream_t stream);
int drpo_normalize(const float* x, const float* mean, const float* std, float eps, float* y, int64_t n, int S,
                   drpo_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DRPO_HIP_H */
