/*
 * vbn_hip.h — C-ABI of the MI355X (gfx950) batched Bayesian-network inference path.
 *
 * Plain pointers and sizes only (no torch types).  All device pointers are HIP device
 * memory; every call is asynchronous on the given hipStream_t (passed as void*).  Return
 * value: 0 on success, otherwise a hipError_t / VBN_E_* code; vbn_hip_last_error() gives
 * the message of the last failure on the calling thread.
 *
 * What each entry point replaces in the reference (Giovannibriglia/VectorizedBayesianNetwork):
 *
 *   vbn_hip_walk            the topological particle pass shared by
 *                             MonteCarloMarginalization.infer_posterior
 *                               (vbn/inference/monte_carlo_marginalization.py:18-92),
 *                             ImportanceSampling.infer_posterior, sampling loop + log-weights
 *                               (vbn/inference/importance_sampling.py:24-80),
 *                             LikelihoodWeighting.infer_posterior
 *                               (vbn/inference/likelihood_weighting.py:24-71),
 *                             _ancestral_sample_tensor (vbn/sampling/ancestral.py:13-41),
 *                           and, through single-step plans with per-particle fixed inputs,
 *                           the per-node BaseCPD.sample / log_prob (vbn/core/base.py:45-59) of
 *                             GaussianNNCPD   (vbn/cpds/gaussian_nn.py:215-288)
 *                             LinearGaussianCPD (vbn/cpds/linear_gaussian.py:163-217)
 *                             MDNCPD          (vbn/cpds/mdn.py:185-272)
 *                             KDECPD          (vbn/cpds/kde.py:105-182)
 *                             SoftmaxNNCPD    (vbn/cpds/softmax_nn.py:581-759).
 *   vbn_hip_posterior_stats VBN._posterior_stats (vbn/vbn.py:483-504), the summary behind
 *                             VBN.infer_relative (vbn/vbn.py:519-568)
 *   vbn_hip_walk (mode GIBBS)  GibbsSampler.sample sweeps (vbn/sampling/gibbs.py:23-92):
 *                             8 candidates per chain drawn by the node's CPD, scored with the
 *                             node's and its children's log-probs, one chosen per chain
 *   vbn_hip_resample        the multinomial resampling step of
 *                             ResampledImportanceSampling._resample
 *                               (vbn/inference/resampled_importance_sampling.py:33-41)
 *   vbn_hip_rb_epilogue     the Rao-Blackwellized mixture / categorical marginal of
 *                             RaoBlackwellizedMarginalization.infer_posterior
 *                               (vbn/inference/rao_blackwellized_marginalization.py:255-317)
 *   vbn_hip_normalize_weights  torch.softmax(log_weights, 1) + ESS
 *                               (importance_sampling.py:82-84) and the normalize / max-shift
 *                               branch of likelihood_weighting.py:75-80.
 */
#ifndef VBN_HIP_H
#define VBN_HIP_H

#ifdef __HIPCC_RTC__               /* runtime compilation of plan-specialised walks (hiprtc) */
using __hip_internal::int32_t;
using __hip_internal::int64_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#else
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define VBN_ABI_VERSION 7

/* error codes besides hipError_t values */
#define VBN_E_ARGS 1001
#define VBN_E_LDS 1002

/* CPD kinds (reference registry keys) */
enum vbn_kind {
  VBN_KIND_GAUSSIAN_NN = 0,
  VBN_KIND_LINEAR_GAUSSIAN = 1,
  VBN_KIND_MDN = 2,
  VBN_KIND_KDE = 3,
  VBN_KIND_SOFTMAX_NN = 4
};

/* role of a node for one query signature */
enum vbn_role {
  VBN_ROLE_SKIP = 0,
  VBN_ROLE_LATENT = 1,
  VBN_ROLE_FIXED = 2,
  VBN_ROLE_PARAMS = 3,  /* write the CPD's conditional parameters, no draw (RB target,
                           CPDHandle.conditional, vbn/core/cpd_handle.py:40-118):
                           gaussian_nn / linear_gaussian: loc[D] ++ scale[D];
                           softmax_nn: class probabilities[D][C];
                           mdn: softmax(logits)[K] ++ loc[K][D] ++ scale[K][D]           */
  VBN_ROLE_SELECT = 4,  /* Gibbs: softmax over the 8 candidate lanes of a chain, choose one,
                           broadcast its value (out_col, out_dim) to the chain's lanes     */
  VBN_ROLE_COLLECT = 5  /* Gibbs: after burn-in, every thin-th sweep, write the target     */
};

/* step flags */
#define VBN_F_LOGP 1        /* add log p(value | parents) to the particle's accumulator */
#define VBN_F_ROOT 2        /* CPD without parents                                        */
#define VBN_F_SHARED 4      /* draws shared across queries (root nodes in MCM/LW/ancestral) */
#define VBN_F_STANDARDIZE 8 /* MLP input (x-mean)/std (gaussian_nn)                          */
#define VBN_F_CLIP 16       /* softmax_nn within_bin_clip                                      */
#define VBN_F_F32L2 32      /* NN CPD: exact f32 MFMA chain for layer 2 instead of split-f16   */
#define VBN_F_KDE_VALU 64   /* kde: pairwise distances on packed VALU (else the 16x16x4 f32 MFMA tile) */
#define VBN_F_KEEP 128      /* fixed role: the value is already in the node's slot (Gibbs)      */
#define VBN_F_LPRESET 256   /* reset the particle's log-prob accumulator before this step       */
#define VBN_F_BM_FIRST 512  /* lean walks: this step's Box-Muller pair also yields the next     */
                            /* VBN_F_BM_SECOND step's dim-0 normal (r sin; this step takes r cos) */
#define VBN_F_BM_SECOND 1024
#define VBN_F_MLP_GENERIC 2048  /* NN CPD with hidden_dims other than (32, 32): every layer as
                                   exact f32 MFMA tiles through LDS; off_w2 points at the layer
                                   table [L, (in, out, off_w, off_b) x L] (int32 in the blob)   */
#define VBN_F_HEAD_MFMA 4096    /* NN CPD head (8..32 outputs) on the split-f16 MFMA like layer 2:
                                   reserved[2] = its fragments [hi 2][64][8 f16] ++ [lo ...]
                                   (1024 floats), then the accumulator-init bias [2][16]      */

/* activations of the NN CPDs (reference gaussian_nn.py:19-24) */
enum vbn_act { VBN_ACT_RELU = 0, VBN_ACT_TANH = 1, VBN_ACT_GELU = 2, VBN_ACT_ELU = 3 };

/* softmax_nn within-bin densities (softmax_nn.py:665-679) */
enum vbn_within { VBN_WITHIN_UNIFORM = 0, VBN_WITHIN_TRIANGULAR = 1, VBN_WITHIN_GAUSSIAN = 2 };

/* engine modes: what happens to the accumulated log-probability at the end */
enum vbn_mode {
  VBN_MODE_MCM = 0,       /* out_lp = exp(lp)          (pdf)          */
  VBN_MODE_WEIGHTED = 1,  /* out_lp = lp               (log-weights)  */
  VBN_MODE_SAMPLE = 2,    /* no out_lp                                */
  VBN_MODE_GIBBS = 3      /* gibbs_iters sweeps over the step table; lane = (chain, candidate),
                             n_samples = 8 candidates; out_x = [B][n_collect][n_out_cols]    */
};

/* One node of the topological walk (32 x int32, filled by the host plan packer).
 * reserved[0] = split-f16 W2 fragments; [1..4] = KDE point packs (NN steps: [1] = the layer-1
 * operand bound zlim as float bits, [2] = the VBN_F_HEAD_MFMA head fragments); [5] = wblk_off, [6] =
 * wblk_len: the NN CPD's weight block [W1 fragments | layer-1/2 accumulator-init biases |
 * split-f16 W2 | W3 | b3], rounded up to a multiple of 256 floats (params float offset,
 * length in floats), which the walk stages into LDS one step ahead (0 = the step runs no
 * MLP); the exact-f32 W2 copy (off_w2) deliberately stays outside the block and is read from
 * global memory on the rare exact path; [7] = one-feature KDE point pack in the
 * v_mfma_f32_32x32x2_f32 operand layout ([rows/32][2][32]: scaled point, |point|^2), or -1. */
typedef struct vbn_step {
  int32_t kind, role, flags, act;
  int32_t n_in, in_off, out_col, out_dim;
  int32_t fixed_col, k, n_out, node_id;
  int32_t noise_idx, aux0, aux1, aux2;
  int32_t off_std, off_w1, off_w2, off_b2, off_w3, off_b3, off_tail, off_pts;
  int32_t reserved[8];
} vbn_step;

/* Arguments of one particle walk over B queries x S samples. */
typedef struct vbn_walk_args {
  const vbn_step* steps;   /* [n_steps] device                                   */
  const int32_t* in_cols;  /* parent column slots, indexed by step.in_off          */
  const float* params;     /* parameter blob                                       */
  const float* fixed;      /* fixed values: [rows][fixed_ld], rows = B or B*S        */
  const float* noise;      /* optional injected draws [n_noise][2][noise_b][S][dmax] */
  const int32_t* out_cols; /* slots written to out_x per particle                   */
  float* out_lp;           /* [B*S] or NULL                                        */
  float* out_x;            /* [B*S][n_out_cols] or NULL                            */
  int64_t n_queries;       /* B                                                    */
  int32_t n_samples;       /* S                                                    */
  int32_t n_steps;
  int32_t n_slots;         /* LDS value slots per particle                          */
  int32_t max_out;         /* widest MLP head (LDS scratch rows)                     */
  int32_t fixed_ld;
  int32_t fixed_per_particle;
  int32_t noise_b;
  int32_t dmax;
  int32_t n_out_cols;
  int32_t mode;            /* enum vbn_mode                                        */
  int32_t kind_mask;       /* CPD kinds walked: 1<<kind, | 32 if a non-relu activation,
                              | 512 if some NN CPD has hidden_dims other than (32, 32) */
  int64_t q_base;          /* global index of query 0 (multi-GPU shards)            */
  uint64_t seed;
  uint64_t offset;         /* RNG stream offset (one per engine call)               */
  float* state;            /* optional particle state [n_slots + 1][B*S] (slot-major; the
                              last row is the log-weight accumulator) for walks split into
                              segments (resampled importance sampling)                 */
  int32_t state_flags;     /* 1: load slots + log-weight from state before the first step;
                              2: store them after the last step                        */
  int32_t gibbs_iters;     /* Gibbs sweeps (mode GIBBS; burn_in + n_collect * thin)   */
  int32_t gibbs_burn_in;
  int32_t gibbs_thin;
  int32_t n_noise;         /* noise nodes per sweep (injected-noise stride, mode GIBBS) */
  int32_t wbuf_floats;     /* >= every step's wblk_len: size of each of the two LDS weight
                              buffers shared by the waves of a workgroup (the caller's
                              contract; torch.ops.vbn_hip.* check it).  When the two buffers
                              do not fit in LDS next to the value slots, the launch runs an
                              unstaged kind set that reads the weights from params      */
  int32_t wave_particles;  /* particles per wave64: 64 (0 = 64) or 32, the half-wave form for
                              launches too small to fill the chip (Gibbs at a few thousand
                              chains): lanes 32-63 mirror lanes 0-31 (same particle and draws,
                              no writes) and the MLPs run one 32-particle MFMA group   */
} vbn_walk_args;

int vbn_hip_abi_version(void);
const char* vbn_hip_last_error(void);
/* sizeof(vbn_walk_args) for which = 0, sizeof(vbn_step) for which = 1 (binding checks) */
int vbn_hip_struct_size(int which);

/* Topological particle walk (see header comment). */
int vbn_hip_walk(const vbn_walk_args* args, void* stream);

/* The kind-set instantiation (walk_inst.hip / VBN_WALK_KIND_SETS: CPD kinds | 64 half-wave |
 * 128 lean | 256 half-wave without injected draws | 512 generic MLP) vbn_hip_walk would launch
 * for these arguments, or -(error code). */
int vbn_hip_walk_kind_set(const vbn_walk_args* args);

/* Plan-specialised walks.  A code object compiled at run time (hiprtc) from
 * csrc/vbn_walk_plan.h for ONE step table and kind set -- the step fields, parent slots and
 * LDS staging schedule as compile-time constants -- is loaded once and launched with the same
 * arguments, grid and LDS as vbn_hip_walk; its outputs are bit-identical to vbn_hip_walk's.
 * vbn_hip_walk_module refuses a launch whose kind set or step count differs from the
 * module's.  (Replaces the same reference call sites as vbn_hip_walk.) */
int vbn_hip_module_load(const void* code_object, const char* kernel_name, uint32_t kind_set, int32_t n_steps,
                        void** handle);
int vbn_hip_walk_module(const void* handle, const vbn_walk_args* args, void* stream);
int vbn_hip_module_unload(void* handle);

/* Per-query weight normalisation over S particles.
 *   normalize=1: w = softmax(log_w) per row, ess[b] = 1/sum(w^2)
 *   normalize=0: w = max(exp(log_w - max(log_w)), eps), ess untouched (may be NULL).
 * log_w and w may alias. */
int vbn_hip_normalize_weights(const float* log_w, float* w, float* ess, int64_t n_queries,
                              int32_t n_samples, int32_t normalize, float eps, void* stream);

/* Multinomial resampling of a segmented walk's particle state (resampled_importance_sampling.py
 * :33-41): per query b, S indices idx[s] ~ Categorical(w[b, :]) (inverse CDF of u[b][s] if u is
 * given, else counter-based Philox keyed by (seed, offset, query q_base + b, s)), then
 * state_out[c][b*S + s] = state_in[c][b*S + idx[s]] for the n_cols - 1 slot rows and
 * state_out[n_cols - 1][.] = 0 (log-weights reset).  state_in and state_out must not alias. */
int vbn_hip_resample(const float* w, const float* u, uint64_t seed, uint64_t offset, int64_t q_base,
                     const float* state_in, float* state_out, int64_t n_queries, int32_t n_samples,
                     int32_t n_cols, void* stream);

/* Weighted posterior summary per query (vbn.py:483-504, _posterior_stats):
 *   w = nan/inf -> 0, clamp >= 0, normalised (uniform 1/S where the sum <= eps);
 *   mean[b][d] = sum_s w x[b][s][d]; std[b][d] = sqrt(max(sum_s w (x - mean)^2, 0));
 *   ess[b] = 1 / max(sum_s w^2, eps).   pdf [B][S], x [B][S][D] contiguous. */
int vbn_hip_posterior_stats(const float* pdf, const float* x, float* mean, float* std, float* ess,
                            int64_t n_queries, int32_t n_samples, int32_t dim, float eps, void* stream);

/* Rao-Blackwellized target epilogue over P particles per query
 * (rao_blackwellized_marginalization.py:68-76, 255-317):
 *   w = normalized weights of log_w (nan -> -1e30, +-inf -> +-1e30, max-shift, exp, sum;
 *       uniform 1/P where the sum <= eps)
 *   mode 0 (gaussian target): params [B][P][2] = (loc, scale); scale sanitized (nan/inf ->
 *       min_scale, abs, >= min_scale); mixture mean/std; grid[b][s] = lo + (hi - lo) z[s] with
 *       lo/hi = mean -+ stddevs std; pdf[b][s] = sum_p w_p N(grid; loc_p, scale_p)
 *   mode 1 (categorical target): params [B][P][C] class probabilities;
 *       pdf[b][c] = sum_p w_p params[b][p][c]  (n_out = C, grid and z unused)
 * params may have a batch of 1 (params_b = 1: shared by every query). */
int vbn_hip_rb_epilogue(const float* log_w, const float* params, int64_t params_b, const float* z,
                        float* pdf, float* grid, int64_t n_queries, int32_t n_particles, int32_t n_out,
                        int32_t mode, float stddevs, float min_scale, float eps, void* stream);

/* LDS bytes of one 64-particle wave's value slots + head scratch (host helper); a workgroup
 * of w waves also holds two weight buffers of wbuf_floats each. */
int64_t vbn_hip_lds_bytes(int32_t n_slots, int32_t max_out);

#ifdef __cplusplus
}
#endif
#endif /* VBN_HIP_H */
