/*
 * vbn_hip_types.h — data layouts shared by the host C-ABI (vbn_hip.h) and the walk kernels:
 * the step table row, the walk arguments, roles, flags and modes.  Kept apart from the entry
 * points so that adding an entry point does not recompile the kernel instantiations.
 */
#ifndef VBN_HIP_TYPES_H
#define VBN_HIP_TYPES_H

#ifdef __HIPCC_RTC__               /* runtime compilation of plan-specialised walks (hiprtc) */
using __hip_internal::int32_t;
using __hip_internal::int64_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#else
#include <stdint.h>
#endif

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
#define VBN_F_PRECOMP 8192      /* per-sample quantities of a node whose parents are all shared
                                   root draws (MCM / LW / ancestral, Q5), computed once per sample
                                   by a one-query pre-pass walk and read from state (state_flags
                                   4; state = the pre-pass out_x [S][stride], aux2 = first column
                                   | stride << 16):  NN CPDs  the n_out MLP head outputs (the MLP
                                   is skipped);  kde (LATENT)  the 16 inverse-CDF chunk sums ++
                                   the underflow shift (pass 1 is skipped)                    */
#define VBN_F_PRE_OUT 16384     /* the pre-pass step of such a node: write those quantities to
                                   out_col .. (NN: n_out, kde: 17 slots) instead of a sample  */
#define VBN_F_PRECOMP_Q 32768   /* with VBN_F_PRECOMP: the quantities are per QUERY -- the node's
                                   parents are all evidence / do values -- computed once per
                                   query by a pre-pass of one wave per query and read from
                                   precomp_q [B][stride] (row b; aux2 as above); needs
                                   n_samples a multiple of 64 (one query per wave)            */

#define VBN_F_CLAMP_EV 65536    /* (ABI v12) fixed role: the value read from the fixed buffer is
                                   clamped as likelihood weighting's clamp_evidence does
                                   (_core.py:112-114): NaN -> 0, then [-1e6, 1e6]            */

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
 * global memory on the rare exact path; [7] = (ABI v12) kde steps: the one-feature moment
 * table of pass 1 (plan.py kde_moment_table: header [u_lo, 1/delta, delta, n_cells] then
 * [n_cells][16 chunks][4 terms] f32), -1 = none; -1 on every other step.  KDE packs [1] (parent features) and
 * [2] (parent ++ target features) hold the bf16x3 slots of v_mfma_f32_16x16x32_bf16
 * ([block][quarter][16 points][8 bf16], plan.py _kde_pack_bf16); [3] = per-point f32 records,
 * [4] = the packed-VALU layout. */
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
  int32_t state_flags;     /* 4 (alone; lean walks): state holds the per-sample quantities of
                              the VBN_F_PRECOMP steps, read-only;
                              1: load slots + log-weight from state before the first step;
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
  const float* precomp_q;  /* (ABI v9) per-query quantities of the VBN_F_PRECOMP_Q steps
                              [B][stride] (read-only; lean walks, n_samples % 64 == 0), or NULL */
  const int32_t* run_if;   /* (ABI v11) device flag or NULL: when *run_if == 0 every wave of the
                              launch returns at once and nothing is written (the importance-
                              sampling -> likelihood-weighting fallback, decided on the device
                              without a host round trip)                                 */
  double* stats_part;      /* (ABI v13) NULL, or the posterior-summary partials of a lean MCM
                              walk (VBN._posterior_stats, vbn/vbn.py:483-504, fused into the
                              walk's epilogue; needs n_samples % 64 == 0, n_out_cols <= 15):
                              per query b and wave k of its S / 64 waves, the row
                              stats_part[(b * S/64 + k) * (2 + 4 D)] of float64
                              [W, Q, then per output column d: m_w, M2_w, m_u, M2_u] with
                              w = pdf nan/inf -> 0 clamped >= 0, W = sum w, Q = sum w^2,
                              m_w = sum w x / W (0 when W = 0), M2_w = sum w (x - m_w)^2,
                              m_u = sum x / 64, M2_u = sum (x - m_u)^2 over the wave's 64
                              particles; vbn_hip_posterior_stats_merge finishes them      */
} vbn_walk_args;

#endif /* VBN_HIP_TYPES_H */
