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
 *                             VBN.infer_relative (vbn/vbn.py:519-568); fused forms (ABI v13):
 *                             the MCM walk's epilogue partials (vbn_walk_args.stats_part) +
 *                             vbn_hip_posterior_stats_merge, and the IS / LW normalisation's
 *                             vbn_hip_normalize_weights_stats
 *   vbn_hip_walk (mode GIBBS)  GibbsSampler.sample sweeps (vbn/sampling/gibbs.py:23-92):
 *                             8 candidates per chain drawn by the node's CPD, scored with the
 *                             node's and its children's log-probs, one chosen per chain
 *   vbn_hip_resample        the multinomial resampling step of
 *                             ResampledImportanceSampling._resample
 *                               (vbn/inference/resampled_importance_sampling.py:33-41)
 *   vbn_hip_rb_epilogue     the Rao-Blackwellized mixture / categorical marginal of
 *                             RaoBlackwellizedMarginalization.infer_posterior
 *                               (vbn/inference/rao_blackwellized_marginalization.py:255-317)
 *   vbn_hip_discrete_posterior  the benchmark adapter's discrete weighted histogram
 *                             _estimate_discrete_posterior[_batch]
 *                               (benchmarking/models/vbn.py:202-242, _normalize_probs 116-121)
 *   vbn_hip_normalize_weights  torch.softmax(log_weights, 1) + ESS
 *                               (importance_sampling.py:82-84) and the normalize / max-shift
 *                               branch of likelihood_weighting.py:75-80.
 */
#ifndef VBN_HIP_H
#define VBN_HIP_H

#include "vbn_hip_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define VBN_ABI_VERSION 13

/* error codes besides hipError_t values */
#define VBN_E_ARGS 1001
#define VBN_E_LDS 1002

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

/* (ABI v8) Mark a loaded module as a Gibbs sweep compiled for chain workgroups of n_waves
 * (1..8) waves (csrc/vbn_walk_plan.h VBN_PLAN_CHAIN_WAVES; the host's phased schedule,
 * vectorizedbayesiannetwork_amd/plan.py gibbs_schedule): vbn_hip_walk_module then launches one
 * workgroup of n_waves waves per 64 (half-wave: 32) candidate lanes, with one LDS copy of their
 * slots (n_slots rows) and n_waves x max(max_out, 1) scratch rows; the waves split each sweep's
 * node updates level by level (and a split level's steps phase by phase).  Same outputs as the
 * sequential sweep, bit for bit.  Only mode GIBBS launches are accepted for such a module; a
 * launch without injected draws may run a module compiled for its kind set | 256 (draw-free).
 * (Replaces the same reference call site as the Gibbs walk: GibbsSampler.sample,
 * vbn/sampling/gibbs.py:36-87.) */
int vbn_hip_module_chain_waves(void* handle, int32_t n_waves);

/* Per-query weight normalisation over S particles.
 *   normalize=1: w = softmax(log_w) per row, ess[b] = 1/sum(w^2)
 *   normalize=0: w = max(exp(log_w - max(log_w)), eps), ess untouched (may be NULL).
 * log_w and w may alias. */
int vbn_hip_normalize_weights(const float* log_w, float* w, float* ess, int64_t n_queries,
                              int32_t n_samples, int32_t normalize, float eps, void* stream);

/* (ABI v11) vbn_hip_normalize_weights with the importance-sampling fallback decision on the
 * device (importance_sampling.py:82-88, no host round trip):
 *   run_if: NULL, or a device flag -- when *run_if == 0 nothing is written (the normalisation of
 *           the predicated likelihood-weighting re-draw, vbn_walk_args.run_if);
 *   flag:   NULL, or a device int32 the caller zeroed: set to 1 when some query's ESS < ess_thr
 *           (NaN ESS never sets it); needs normalize = 1. */
int vbn_hip_normalize_weights_ex(const float* log_w, float* w, float* ess, int64_t n_queries, int32_t n_samples,
                                 int32_t normalize, float eps, const int32_t* run_if, int32_t* flag, float ess_thr,
                                 void* stream);

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

/* (ABI v13) The same summary finished from a lean MCM walk's epilogue partials
 * (vbn_walk_args.stats_part, n_parts = S / 64 rows of 2 + 4 dim doubles per query): Chan's merge
 * of the waves' (W, m_w, M2_w) -- or of (64, m_u, M2_u) where W <= eps, the reference's uniform
 * weights -- in float64; mean / std [B][dim], ess [B] float32 as vbn_hip_posterior_stats. */
int vbn_hip_posterior_stats_merge(const double* part, int64_t n_queries, int32_t n_parts, int32_t dim, float eps,
                                  float* mean, float* std, float* ess, void* stream);

/* (ABI v13) vbn_hip_normalize_weights_ex with the posterior summary of the weights it writes
 * fused into the same pass (importance_sampling.py:82-84 / likelihood_weighting.py:75-80, then
 * vbn.py:483-504 on (w, x)): the row stays in registers, x [B][S][dim] is read once more for
 * the centred second moment.  mean / std [B][dim], stats_ess [B]; stats_eps is
 * _posterior_stats' eps.  Needs n_samples <= 4096 (else VBN_E_ARGS: use the two calls). */
int vbn_hip_normalize_weights_stats(const float* log_w, float* w, float* ess, int64_t n_queries, int32_t n_samples,
                                    int32_t normalize, float eps, const int32_t* run_if, int32_t* flag,
                                    float ess_thr, const float* x, int32_t dim, float stats_eps, float* mean,
                                    float* std, float* stats_ess, void* stream);

/* (ABI v10) Discrete weighted histogram per query (benchmarking/models/vbn.py:202-242):
 *   for s in order: skip a non-finite w[b][s]; i = rint(x[b][s]) (half to even); skip i
 *   outside [0, k); bins[i] += (double)w[b][s]  (float64 running sums, the reference's order);
 *   probs[b][c] = bins[c] / total with total = numpy's pairwise sum of the bins, or 1/k each
 *   when total is not finite or <= 0 (_normalize_probs, vbn.py:116-121).
 *   bad[b] = 0, or 1 / 2 when a finite-weight sample is NaN / +-inf (the reference raises
 *   ValueError / OverflowError there; that query's probs are then not meaningful).
 *   x: sample s of query b at x[(b * n_samples + s) * x_stride] (x_stride = D of a [B][S][D]
 *   tensor: feature 0); w [B][S]; probs [B][k] float64; bad [B] int32. */
int vbn_hip_discrete_posterior(const float* x, int64_t x_stride, const float* w, double* probs, int32_t* bad,
                               int64_t n_queries, int32_t n_samples, int32_t k, void* stream);

/* (ABI v11) vbn_hip_discrete_posterior for float32 or float64 samples / weights (x_f64, w_f64:
 * 0 = float32, 1 = float64).  The reference converts each element with float() before it bins
 * or sums it, so a float64 input is binned and summed at its own precision. */
int vbn_hip_discrete_posterior_typed(const void* x, int32_t x_f64, int64_t x_stride, const void* w, int32_t w_f64,
                                     double* probs, int32_t* bad, int64_t n_queries, int32_t n_samples, int32_t k,
                                     void* stream);

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
