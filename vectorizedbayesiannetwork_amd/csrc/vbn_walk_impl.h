#pragma once
// vbn_walk_impl.h — gfx950 (MI355X) particle walk for batched Bayesian-network inference:
// the device code and the vbn_walk_kernel template, shared by vbn_walk.hip (host entry points)
// and walk_inst.hip (one kind-set instantiation per object, built in parallel).
//
// One wave64 owns 64 particles (lane == particle in every per-particle stage).  The wave
// walks the plan's topological steps; each node's value lives in LDS (vals[slot][64]), so
// the [B,S,sum(D)] particle tensor of the reference never touches HBM: only evidence in,
// pdf/log-weights and the target slice out.
//
// NN CPDs (gaussian_nn, mdn, softmax_nn; MLP in->32->32->out): the 32x32 hidden layer runs
// on MFMA (v_mfma_f32_32x32x2_f32, exact f32) with the hidden unit on the M axis and the
// particle on the N axis, two 32-particle groups per wave.  Layer 1 (K = #parents <= few)
// is computed on VALU directly in the MFMA B-operand layout, the head on VALU from the
// accumulator layout, combined across lane halves with one v_permlane32_swap per output.
//
// Reference ops replaced (file:line in Giovannibriglia/VectorizedBayesianNetwork):
//   topo loop            vbn/inference/monte_carlo_marginalization.py:60-91,
//                        importance_sampling.py:56-80, likelihood_weighting.py:41-71,
//                        vbn/sampling/ancestral.py:26-40
//   gaussian_nn          vbn/cpds/gaussian_nn.py:215-288
//   linear_gaussian      vbn/cpds/linear_gaussian.py:163-217
//   mdn                  vbn/cpds/mdn.py:185-272
//   kde                  vbn/cpds/kde.py:105-182
//   softmax_nn           vbn/cpds/softmax_nn.py:581-759
//   softmax + ESS        importance_sampling.py:82-84, likelihood_weighting.py:75-80
#ifndef __HIPCC_RTC__               // hiprtc (plan-specialised walks) brings its own runtime
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#endif

#include "vbn_hip_types.h"

#ifndef INFINITY
#define INFINITY __builtin_inff()
#endif

#define WAVE 64
#define KDE_CHUNKS 16
// kde steps: blob offset of the one-feature moment table (plan.kde_moment_table), -1 = none
#define KDE_MT(st) ((st).reserved[7])
#define KDE_REC_TAIL 16  // weight-0 record rows after the last point (plan.py KDE_REC_TAIL)
#define LOG_2PI_F 1.8378770664093453f

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// step field holding the split-f16 W2 fragments (vbn_step.reserved[0])
#define OFF_W2H(st) ((st).reserved[0])

// ------------------------------------------------------------------------------------------
// small device helpers
// ------------------------------------------------------------------------------------------

__device__ __forceinline__ void wave_sync() {
  // LDS ops of one wave are issued in order; this only stops the compiler from moving
  // LDS accesses of different lanes across the hand-off point.
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_wave_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// relu as one v_max_i32 on the float's bits (negative floats are negative ints; -0 -> +0).
// fmaxf would add a canonicalising v_max(x, x) in IEEE mode, inline asm would hide the
// MFMA->VALU read hazard from the compiler.  NaN parents are handled by the caller.
__device__ __forceinline__ float relu_nan(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

template <int ACT>
__device__ __forceinline__ float act_fn(float x) {
  if (ACT == VBN_ACT_RELU) return relu_nan(x);
  if (ACT == VBN_ACT_TANH) return tanhf(x);
  if (ACT == VBN_ACT_GELU) return x * 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
  return x > 0.f ? x : expm1f(x);  // ELU(alpha=1)
}

// Hardware transcendentals without the library's denormal / correctly-rounded fix-ups: the
// natural log as v_log_f32 (log2) x ln 2 and the reciprocal as v_rcp_f32 (each ~1 ulp).  Only
// for arguments that are normal floats by construction (the callers say why): __logf /
// __fdividef / sqrtf lower to ~12-instruction sequences that handle denormal inputs, which
// was ~10 % of the cfg2 walk's VALU stream (softplus and Box-Muller once per node).
#define VBN_LN2_F 0.69314718055994530942f
__device__ __forceinline__ float log_hw(float x) { return __builtin_amdgcn_logf(x) * VBN_LN2_F; }

// F.softplus(beta=1, threshold=20) (reference cpds/utils.py:6-7) with hardware exp/log:
// log1p(e) as Kahan's log(u) * e / (u - 1) (u - 1 is exact) for x >= -5 (u in [1, 2^29]:
// normal), a 4-term series below (relative error < 1e-9 there).
__device__ __forceinline__ float softplus_t(float x) {
#ifdef VBN_ABL_NOSOFTPLUS
  return x;
#endif
  if (x > 20.f) return x;
  const float e = __expf(x);
  if (x < -5.f) return e * (1.f - e * (0.5f - e * (0.33333334f - e * 0.25f)));
  const float u = 1.0f + e;
  return log_hw(u) * (e * __builtin_amdgcn_rcpf(u - 1.0f));   // u - 1 >= e^-5: normal
}

// Philox-2x32-10 counter-based RNG (Random123): counter (c0, c1), 32-bit key; one
// v_mad_u64_u32 and one three-input XOR (gfx950 v_bitop3_b32, truth table 0x96) per round.
__device__ __forceinline__ uint2 philox2x32(uint2 c, uint32_t k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p = (uint64_t)0xD256D193u * c.x;
    c = make_uint2(__builtin_amdgcn_bitop3_b32((uint32_t)(p >> 32), k, c.y, 0x96), (uint32_t)p);
    k += 0x9E3779B9u;
  }
  return c;
}

__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// r = sqrt(-2 ln u1) with u1 in [2^-24, 1] (normal) on v_log_f32 / v_sqrt_f32 (-2 ln u1 in
// [0, 33.3]: normal or 0)
__device__ __forceinline__ float bm_radius(float u1) {
  return __builtin_amdgcn_sqrtf(-2.0f * log_hw(u1));
}

__device__ __forceinline__ float box_muller(uint32_t a, uint32_t b) {
  const float u1 = (float)((a >> 8) + 1u) * (1.0f / 16777216.0f);  // (0,1]
  const float u2 = (float)(b >> 8) * (1.0f / 16777216.0f);
  return bm_radius(u1) * __builtin_amdgcn_cosf(u2);                 // cos(2*pi*u2)
}

struct Lane {
  const float* P;        // parameter blob (from a __restrict__ kernel argument)
  const int32_t* ic;     // parent column slots (from a __restrict__ kernel argument)
  float* vals;   // LDS [n_slots][64]
  float* scr;    // LDS [max_out][64]
  const float* wb;  // LDS: this step's weight block (wblk, staged one step ahead by the workgroup)
  int lane;
  int64_t p;     // particle (clamped)
  int64_t b;     // query (Gibbs: chain)
  int s;         // sample (Gibbs: candidate)
  int iter;      // Gibbs sweep (0 for every other walk)
  bool valid;    // particle index inside the batch
  bool mirror;   // half-wave launch: lanes 32-63 mirror lanes 0-31 (kind-set bit 6)
  bool lean;     // no injected draws, no segment state, not Gibbs (kind-set bit 7): the
                 // kernel sets these from KM, so every inlined check on them folds away
  bool noiseless;  // no injected draws (lean, or kind-set bit 8: production Gibbs)
  bool wq;       // every lane of the wave is in the same query (S a multiple of the wave's particles)
  mutable float bm_spare;  // lean walks: the r sin half of a VBN_F_BM_FIRST step's Box-Muller pair
};

// Draws of node ``st``, dimension d, for this particle.  Stream 0 gives a standard normal
// (Box-Muller on both words), stream 1 two uniforms: the categorical / index choice and the
// within-bin uniform, stream 2 the Gibbs chain choice (one per chain and sweep).  Counter =
// (sample, query ^ seed_hi), key = seed_lo + stream id, where the query key is 0 for draws
// shared by all queries (root nodes in MCM/LW/ancestral, Q5).  Stream id = offset[8] |
// node[14] | dim[8] | stream[2]: disjoint for every (node, dim, stream) the host admits
// (PackedModel: < 16384 nodes, < 256 dims per node).
// With injected noise (parity tests) slot 0 = categorical uniform, slot 1 = normal / uniform.
#define RNG_NORMAL 0
#define RNG_UNIFORM 1
#define RNG_SELECT 2
__device__ __forceinline__ uint2 rng_words(const vbn_walk_args& A, const vbn_step& st, int d, int stream,
                                           const Lane& L) {
  const uint32_t qkey = (st.flags & VBN_F_SHARED) ? 0u : (uint32_t)(A.q_base + L.b + 1);
  const uint32_t sid = ((uint32_t)(A.offset & 0xffu) << 24) | ((uint32_t)st.node_id << 10) |
                       ((uint32_t)d << 2) | (uint32_t)stream;
  const uint32_t ctr = (uint32_t)L.s + (uint32_t)L.iter * (uint32_t)A.n_samples;
  return philox2x32(make_uint2(ctr, qkey ^ (uint32_t)(A.seed >> 32)), (uint32_t)A.seed + sid);
}

__device__ __forceinline__ int64_t noise_index(const vbn_walk_args& A, const vbn_step& st, int d, int slot,
                                               const Lane& L) {
  const int64_t bq = A.noise_b == 1 ? 0 : L.b;
  const int64_t stride_slot = (int64_t)A.noise_b * A.n_samples * A.dmax;
  const int64_t stride_iter = (int64_t)A.n_noise * 2 * stride_slot;       // Gibbs sweeps
  return (int64_t)L.iter * stride_iter + ((int64_t)st.noise_idx * 2 + slot) * stride_slot +
         (bq * A.n_samples + L.s) * A.dmax + d;
}

__device__ __forceinline__ float draw_normal(const vbn_walk_args& A, const vbn_step& st, int d, const Lane& L) {
  if (!L.noiseless && A.noise) return A.noise[noise_index(A, st, d, 1, L)];
#ifdef VBN_ABL_NORNG
  return 0.5f;
#endif
  // lean walks pair the dim-0 normals of consecutive one-dimensional gaussian steps (host flags,
  // plan.py _pair_normals): the first step's Philox pair gives r cos(2 pi u2) to itself and
  // r sin(2 pi u2) -- an independent N(0, 1) -- to the second, halving Philox + log + sqrt
  if (L.lean && d == 0 && (st.flags & VBN_F_BM_SECOND)) return L.bm_spare;
  const uint2 w = rng_words(A, st, d, RNG_NORMAL, L);
  if (L.lean && d == 0 && (st.flags & VBN_F_BM_FIRST)) {
    const float u1 = (float)((w.x >> 8) + 1u) * (1.0f / 16777216.0f);
    const float u2 = (float)(w.y >> 8) * (1.0f / 16777216.0f);
    const float r = bm_radius(u1);
    L.bm_spare = r * __builtin_amdgcn_sinf(u2);
    return r * __builtin_amdgcn_cosf(u2);
  }
  return box_muller(w.x, w.y);
}

// (categorical uniform, within-bin uniform)
__device__ __forceinline__ float2 draw_uniforms(const vbn_walk_args& A, const vbn_step& st, int d, const Lane& L) {
  if (!L.noiseless && A.noise)
    return make_float2(A.noise[noise_index(A, st, d, 0, L)], A.noise[noise_index(A, st, d, 1, L)]);
  const uint2 w = rng_words(A, st, d, RNG_UNIFORM, L);
  return make_float2(u01(w.x), u01(w.y));
}

// Read-only buffers (parameter blob, slot lists, evidence) seen through the constant address
// space: wave-uniform reads become scalar loads (s_load, lgkmcnt) instead of vector loads.
typedef __attribute__((address_space(4))) const float cfloat;
typedef __attribute__((address_space(4))) const int32_t cint;
#define CP(p) ((cfloat*)(p))
#define CI(p) ((cint*)(p))

__device__ __forceinline__ float vread(const Lane& L, int slot) { return L.vals[slot * WAVE + L.lane]; }
__device__ __forceinline__ void vwrite(const Lane& L, int slot, float v) { L.vals[slot * WAVE + L.lane] = v; }

__device__ __forceinline__ float fixed_value(const vbn_walk_args& A, const vbn_step& st, int d,
                                             const Lane& L) {
  if (!A.fixed_per_particle && L.wq) {               // one query per wave: a scalar load
    const int64_t b = ((int64_t)__builtin_amdgcn_readfirstlane((int)(L.b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((int)L.b);
    return CP(A.fixed)[b * A.fixed_ld + st.fixed_col + d];
  }
  const int64_t row = A.fixed_per_particle ? L.p : L.b;
  return A.fixed[row * A.fixed_ld + st.fixed_col + d];
}

// likelihood weighting's clamp_evidence (_core.py:112-114) on the value read, for steps with
// VBN_F_CLAMP_EV: the unclamped fixed buffer of importance sampling serves its fallback as is
__device__ __forceinline__ float fixed_read(const vbn_walk_args& A, const vbn_step& st, int d, const Lane& L) {
  const float v = fixed_value(A, st, d, L);
  if (st.flags & VBN_F_CLAMP_EV) return v != v ? 0.f : fminf(fmaxf(v, -1e6f), 1e6f);
  return v;
}

// VBN_F_PRECOMP: this sample's row of the node's pre-pass quantities (state_flags 4: state =
// the one-query pre-pass walk's out_x [S][stride]; aux2 = first column | stride << 16)
__device__ __forceinline__ const float* precomp_row(const vbn_walk_args& A, const vbn_step& st, const Lane& L) {
  const int col = st.aux2 & 0xffff, stride = (int)((unsigned)st.aux2 >> 16);
  return A.state + (int64_t)L.s * stride + col;
}

// VBN_F_PRECOMP | VBN_F_PRECOMP_Q: this query's row of the per-query pre-pass quantities
// (precomp_q [B][stride]); one query per wave (host: n_samples % 64 == 0), so the row address is
// wave-uniform and its reads are scalar loads
__device__ __forceinline__ const cfloat* precomp_qrow(const vbn_walk_args& A, const vbn_step& st, const Lane& L) {
  const int col = st.aux2 & 0xffff, stride = (int)((unsigned)st.aux2 >> 16);
  const int64_t b = ((int64_t)__builtin_amdgcn_readfirstlane((int)(L.b >> 32)) << 32) |
                    (uint32_t)__builtin_amdgcn_readfirstlane((int)L.b);
  return CP(A.precomp_q) + b * stride + col;
}

// value of a fixed node: from the fixed buffer, or (VBN_F_KEEP, Gibbs) the slot's current value
__device__ __forceinline__ float node_fixed(const vbn_walk_args& A, const vbn_step& st, int d,
                                            const Lane& L) {
  return (!L.lean && (st.flags & VBN_F_KEEP)) ? vread(L, st.out_col + d) : fixed_read(A, st, d, L);
}

// ------------------------------------------------------------------------------------------
// MLP (in -> 32 -> 32 -> n_out) for the wave's 64 particles; head outputs to scr[j][lane].
//
// Two 32-particle groups per wave (g = 0: particles 0-31, g = 1: 32-63).  Both hidden layers
// run with the hidden unit on M and the particle on N; both accumulators start from the layer's
// bias (register r of lane half h = b[row(r, h)], four 16-byte loads, exact f32).
//   layer 1: K = n_in on v_mfma_f32_32x32x2_f32, A = W1 fragments, B = z of the lane's particle
//   layer 2: K = 32 on v_mfma_f32_32x32x16_f16 as a 3-pass split product: x = hi + lo with
//            hi = f16(x), lo = f16(x - hi) for both operands; A_lo.B_hi + A_hi.B_lo + A_hi.B_hi
//            accumulated in f32 (relative error ~2^-22 per product, i.e. fp32-level) at 1/5
//            of the f32-MFMA time.  The layer-1 accumulator IS the B operand: register 8s+j
//            of lane half h holds hidden row 16s + 8(j>>2) + 4h + (j&3), and the host packs
//            W2 in that k order.  If any |h| > 32768 (f16 range) the wave takes the exact
//            f32 chain (v_mfma_f32_32x32x2_f32, k-step s pairs rows (row(s,0), row(s,1))).
//   head   : 16 v_permlane32_swap transpose the layer-2 accumulators so lane l holds all 32
//            hidden units of particle l; the head then runs on VALU with wave-uniform weights.
//
// Parameter blocks (packed by vectorizedbayesiannetwork_amd/plan.py):
//   off_std : mean_x[n_in], 1/std_x[n_in]                            (gaussian_nn only)
//   off_w1  : [t][64]  lane l: W1z[l&31][2t + (l>>5)],  W1z = [W1 | 0] (even width)
//   off_b2  : [layer 2][group 2][half 2][16] = b[row(r, h)] (accumulator init; the two group
//             copies are identical)
//   off_w2  : [q 4][lane 64][4], step s = 4q+e: W2[l&31][row(s, l>>5)]   (exact f32 fallback)
//   off_w2h : [4][lane 64][8 f16]: hi(s=0), hi(s=1), lo(s=0), lo(s=1);
//             element j of lane l: W2[l&31][16s + 8(j>>2) + 4(l>>5) + (j&3)]
//   off_w3  : [n_out][32] = W3[j][row(r,0)] (r<16) ++ W3[j][row(r,1)]
//   off_b3  : [n_out]
// with row(r, h) = (r&3) + 8(r>>2) + 4h, the 32x32 accumulator row of register r, half h.
// ------------------------------------------------------------------------------------------

// layer-1 B operand of k-step t for group g: z[2t + half] of particle (c + 32 g); the
// column beyond n_in (odd n_in) is 0.
// The operands of both lane halves are read with wave-uniform addresses (scalar loads) and
// selected per lane: a per-lane address would make them vector loads, whose vmcnt wait also
// waits for the next step's weight-block DMA.
template <bool STD, int NIN>
__device__ __forceinline__ float l1_operand(const vbn_walk_args& A, const vbn_step& st, const Lane& L,
                                            int t, int g) {
  const int half = L.lane >> 5;
  const int nin = NIN > 0 ? NIN : st.n_in;
  const int kk = 2 * t + half;
  const int ke = min(2 * t, nin - 1), ko = min(2 * t + 1, nin - 1);
  const int se = CI(L.ic)[st.in_off + ke], so = CI(L.ic)[st.in_off + ko];
  const int slot = half ? so : se;
  float z = L.vals[slot * WAVE + (L.lane & 31) + 32 * g];
  if (STD) {
    const cfloat* sp = CP(L.P) + st.off_std;
    const float me = sp[ke], mo = sp[ko], ie = sp[nin + ke], io = sp[nin + ko];
    z = (z - (half ? mo : me)) * (half ? io : ie);
  }
  return kk < nin ? z : 0.0f;
}

#define WBLK_OFF(st) ((st).reserved[5])
#define WBLK_LEN(st) ((st).reserved[6])

// Layer-1 accumulator init of group g = bias rows of the lane half (register r of half h =
// b1[row(r, h)]), from the staged weight block (LDS) or, on the exact fallback, the blob.
__device__ __forceinline__ f32x16 load_acc16(const float* __restrict__ src) {
  const float4* q4 = reinterpret_cast<const float4*>(src);
  f32x16 a;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 v = q4[q];
    a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
  }
  return a;
}

// layer-2 bias as the accumulator's initial value of group g (exact f32 fallback path)
__device__ __forceinline__ f32x16 layer2_init(const vbn_step& st, const Lane& L, int g) {
  const float4* bacc = reinterpret_cast<const float4*>(L.P + st.off_b2 + 64 + 32 * g + 16 * (L.lane >> 5));
  f32x16 b;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 v = bacc[q];
    b[4 * q] = v.x; b[4 * q + 1] = v.y; b[4 * q + 2] = v.z; b[4 * q + 3] = v.w;
  }
  return b;
}

// y - f32(half h of packed f16 pair ph), exact: one v_fma_mix_f32 (reads the f16 in place),
// selected by the compiler from fma(f32(h), m, y) with m = -1 held opaque in an SGPR (a literal
// -1 folds the fma into a subtraction, which gfx950 selects as cvt + sub).  Not inline asm: an
// asm v_fma_mix is invisible to the hazard recognizer, which then does not pad its VGPR write
// against an in-flight MFMA reading or writing that register -- the cause of round 3's
// hipcc / hiprtc divergence of the split-f16 heads (the two compiles scheduled it differently).
__device__ __forceinline__ float neg_one_sgpr() {
  float m = -1.0f;
  asm("" : "+s"(m));     // not volatile: CSE'd / hoisted like any pure value
  return m;
}
__device__ __forceinline__ float sub_f16_lo(float y, f16x2 ph) {
  return __builtin_fmaf((float)ph[0], neg_one_sgpr(), y);
}
__device__ __forceinline__ float sub_f16_hi(float y, f16x2 ph) {
  return __builtin_fmaf((float)ph[1], neg_one_sgpr(), y);
}

// Layer 2 of one group on the split-f16 path from the activations y (|y| <= 32768 checked by
// the caller): y = hi + lo with hi = f16(y), lo = f16(y - hi); A_lo.B_hi + A_hi.B_lo + A_hi.B_hi
// on v_mfma_f32_32x32x16_f16 (f32 accumulate).  B operand: register 8s+j of lane half h holds
// hidden row 16s + 8(j>>2) + 4h + (j&3).
__device__ __forceinline__ f32x16 layer2_split(const uint4 (&w2h)[4], const f32x16& binit, const float (&y)[16]) {
#ifdef VBN_ABL_NOL2
  f32x16 r = binit;
  for (int i = 0; i < 16; ++i) r[i] += y[i];
  return r;
#endif
  f16x8 bh[2], bl[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const float y0 = y[8 * s2 + j], y1 = y[8 * s2 + j + 1];
      const f16x2 ph = __builtin_convertvector((f32x2){y0, y1}, f16x2);
#ifdef VBN_ABL_NOSPLIT
      const f16x2 pl = ph;
#else
      const f16x2 pl = __builtin_convertvector((f32x2){sub_f16_lo(y0, ph), sub_f16_hi(y1, ph)}, f16x2);
#endif
      bh[s2][j] = ph[0];
      bh[s2][j + 1] = ph[1];
      bl[s2][j] = pl[0];
      bl[s2][j + 1] = pl[1];
    }
  }
  f32x16 b = binit;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const f16x8 ah = __builtin_bit_cast(f16x8, w2h[s2]);
    const f16x8 al = __builtin_bit_cast(f16x8, w2h[2 + s2]);
#ifndef VBN_ABL_NOSPLIT
    b = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s2], b, 0, 0, 0);
    b = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s2], b, 0, 0, 0);
#endif
    b = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s2], b, 0, 0, 0);
  }
  return b;
}

// Layer 2 of one group from the raw layer-1 pre-activations z with the ReLU folded into the
// f16 split (the caller guarantees z < 2048): hi = f16 of z rounded toward zero, so the
// residual z - hi lies in [0, 1) for z >= 0 and in (-1, 0] for z < 0; one v_fma_mix_f32 with
// the clamp bit ([0, 1]) then gives relu(z) - relu(hi) exactly, and one v_pk_max_f16 per pair
// gives relu(hi): hi + lo = relu(z) to f16 x f16 precision, 5 VALU per pair of activations
// instead of 6 (two ReLU maxes, two conversions, two residuals).
__device__ __forceinline__ f32x16 layer2_split_relu(const uint4 (&w2h)[4], const f32x16& binit,
                                                    const float (&z)[16]) {
  f16x8 bh[2], bl[2];
  const f16x2 zero2 = {(_Float16)0.f, (_Float16)0.f};
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const float z0 = z[8 * s2 + j], z1 = z[8 * s2 + j + 1];
      const f16x2 pr = __builtin_bit_cast(f16x2, __builtin_amdgcn_cvt_pkrtz(z0, z1));
      const float r0 = __builtin_amdgcn_fmed3f(sub_f16_lo(z0, pr), 0.f, 1.f);
      const float r1 = __builtin_amdgcn_fmed3f(sub_f16_hi(z1, pr), 0.f, 1.f);
      const f16x2 pl = __builtin_convertvector((f32x2){r0, r1}, f16x2);
      const f16x2 ph = __builtin_elementwise_max(pr, zero2);
      bh[s2][j] = ph[0];
      bh[s2][j + 1] = ph[1];
      bl[s2][j] = pl[0];
      bl[s2][j + 1] = pl[1];
    }
  }
  f32x16 b = binit;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const f16x8 ah = __builtin_bit_cast(f16x8, w2h[s2]);
    const f16x8 al = __builtin_bit_cast(f16x8, w2h[2 + s2]);
    b = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s2], b, 0, 0, 0);
    b = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s2], b, 0, 0, 0);
    b = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s2], b, 0, 0, 0);
  }
  return b;
}

// Layer 2 of one group from the activations y, exact f32 chain (K = 32 as 16
// v_mfma_f32_32x32x2_f32 steps)
__device__ __forceinline__ f32x16 layer2_exact(const vbn_step& st, const Lane& L, int g, const float (&y)[16]) {
  const float4* w2p = reinterpret_cast<const float4*>(L.P + st.off_w2);
  f32x16 b = layer2_init(st, L, g);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 v = w2p[q * WAVE + L.lane];
    b = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, y[4 * q + 0], b, 0, 0, 0);
    b = __builtin_amdgcn_mfma_f32_32x32x2f32(v.y, y[4 * q + 1], b, 0, 0, 0);
    b = __builtin_amdgcn_mfma_f32_32x32x2f32(v.z, y[4 * q + 2], b, 0, 0, 0);
    b = __builtin_amdgcn_mfma_f32_32x32x2f32(v.w, y[4 * q + 3], b, 0, 0, 0);
  }
  return b;
}

// Head outputs two at a time (both outputs' weights in flight together; w3/b3 (weight block)
// and scr (head scratch) are distinct LDS rows, so the reads need not wait for the writes).
__device__ __forceinline__ float head_dot(const float4 (&w)[4], const float (&y0)[16], const float (&y1)[16],
                                          float b, bool nan_in) {
  float a0 = 0.f, c0 = 0.f, a1 = 0.f, c1 = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    a0 = fmaf(w[q].x, y0[4 * q], a0);
    c0 = fmaf(w[q].y, y0[4 * q + 1], c0);
    a1 = fmaf(w[q].x, y1[4 * q], a1);
    c1 = fmaf(w[q].y, y1[4 * q + 1], c1);
    a0 = fmaf(w[q].z, y0[4 * q + 2], a0);
    c0 = fmaf(w[q].w, y0[4 * q + 3], c0);
    a1 = fmaf(w[q].z, y1[4 * q + 2], a1);
    c1 = fmaf(w[q].w, y1[4 * q + 3], c1);
  }
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0 + c0), __float_as_uint(a1 + c1), false, false);
  const float o = (__uint_as_float(sw[0]) + __uint_as_float(sw[1])) + b;
  return nan_in ? __int_as_float(0x7fc00000) : o;
}

__device__ __forceinline__ void head_outputs(const float* __restrict__ w3, const float* __restrict__ b3,
                                             float* __restrict__ scr, int nout, const float (&y0)[16],
                                             const float (&y1)[16], bool nan_in) {
#pragma clang loop unroll(disable)
  for (int j = 0; j < nout; j += 2) {
    const bool two = j + 1 < nout;
    const float4* wa = reinterpret_cast<const float4*>(w3 + 32 * j);
    const float4* wb = reinterpret_cast<const float4*>(w3 + 32 * (two ? j + 1 : j));
    const float4 va[4] = {wa[0], wa[1], wa[2], wa[3]};
    const float4 vb[4] = {wb[0], wb[1], wb[2], wb[3]};
    const float ba = b3[j], bb = b3[two ? j + 1 : j];
    scr[j * WAVE] = head_dot(va, y0, y1, ba, nan_in);
    if (two) scr[(j + 1) * WAVE] = head_dot(vb, y0, y1, bb, nan_in);
  }
}

// Head on VALU in the accumulator layout (no transpose): lane half h holds hidden rows
// row(r, h) of its particle, so per output j the half's 16 products use per-lane weights
// W3[j][row(r, h)] (the pack's [n_out][32] rows hold 16 per half), in two independent chains
// per group; one v_permlane32_swap per output then adds the two halves (group 0 | group 1 ->
// lane l = particle l).  W = the step's weight block (W3 at off_w3, b3 at off_b3, relative to
// wblk_off); outputs to scr[j][lane].
template <int ACT>
__device__ __forceinline__ void mlp_head(const vbn_step& st, const Lane& L, const float* __restrict__ W,
                                         const f32x16& h0, const f32x16& h1, bool nan_in) {
  const int lane = L.lane;
#ifdef VBN_ABL_NOHEAD
  for (int j = 0; j < st.n_out; ++j) L.scr[j * WAVE + lane] = h0[j] + h1[j + 1];
  wave_sync();
  return;
#endif
  float y0[16], y1[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    y0[r] = act_fn<ACT>(h0[r]);
    y1[r] = act_fn<ACT>(h1[r]);
  }
  head_outputs(W + (st.off_w3 - WBLK_OFF(st)) + 16 * (lane >> 5), W + (st.off_b3 - WBLK_OFF(st)),
               L.scr + lane, st.n_out, y0, y1, nan_in);
  wave_sync();
}

// Layer 1 of group g (v_mfma_f32_32x32x2_f32, K = n_in, bias rows as the accumulator init)
// and its activation.  W = weight block base (LDS: staged block; global: blob + wblk_off), so
// W1 sits at W[t * 64 + lane] and the biases at W + (off_b2 - wblk_off).  ``pre`` runs between
// the fragment reads and the first MFMA (group 0: the step's draws).  Returns a wave-uniform
// flag: CHK = 0 (fast path) -- some layer-1 operand lies beyond the node's bound zlim
// (VBN_ZLIM: within it no activation can leave the f16 split range, plan._pack_mlp), one
// compare per MFMA operand instead of one max per activation; CHK = 1 -- some activation
// leaves the split range |y| <= 32768 (NaN with the sign bit clear counts as out of range).
#define VBN_ZLIM(st) __int_as_float((st).reserved[1])
template <int ACT, bool STD, int NIN, int CHK = 0, bool RAW = false, typename F>
__device__ __forceinline__ bool mlp_l1_act(const vbn_walk_args& A, const vbn_step& st, const Lane& L,
                                           const float* __restrict__ W, int g, float (&y)[16], F&& pre) {
  const int lane = L.lane;
  f32x16 a = load_acc16(W + (st.off_b2 - WBLK_OFF(st)) + 32 * g + 16 * (lane >> 5));
  const float zlim = VBN_ZLIM(st);
  bool out = false;
  if (NIN > 0) {
    float w1[(NIN + 1) / 2 > 0 ? (NIN + 1) / 2 : 1];
#pragma unroll
    for (int t = 0; t < (NIN + 1) / 2; ++t) w1[t] = W[t * WAVE + lane];
    pre();
#pragma unroll
    for (int t = 0; t < (NIN + 1) / 2; ++t) {
      const float op = l1_operand<STD, NIN>(A, st, L, t, g);
      if (CHK == 0) out |= !(fabsf(op) <= zlim);
      a = __builtin_amdgcn_mfma_f32_32x32x2f32(w1[t], op, a, 0, 0, 0);
    }
  } else {
    pre();
    const int t1 = (st.n_in + 1) >> 1;
    for (int t = 0; t < t1; ++t) {
      const float op = l1_operand<STD, NIN>(A, st, L, t, g);
      if (CHK == 0) out |= !(fabsf(op) <= zlim);
      a = __builtin_amdgcn_mfma_f32_32x32x2f32(W[t * WAVE + lane], op, a, 0, 0, 0);
    }
  }
  int big = 0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    y[r] = RAW ? a[r] : act_fn<ACT>(a[r]);                // RAW: relu folded into the split
    if (CHK == 1) big = max(big, __float_as_int(y[r]));   // activations are >= -1: the positive side
  }
  // split range: relu nodes (layer2_split_relu) z < 2048, others |act(z)| <= 32768
  return CHK == 1 ? __any(big > (ACT == VBN_ACT_RELU ? 0x44ffffff : 0x47000000)) : __any(out);
}

// Head outputs with a compile-time count (NOUT > 0): straight-line code, so the scheduler can
// place it beside the other group's layer-2 MFMAs (same operations as head_outputs).
template <int NOUT>
__device__ __forceinline__ void head_outputs_n(const float* __restrict__ w3, const float* __restrict__ b3,
                                               float* __restrict__ scr, const float (&y0)[16],
                                               const float (&y1)[16], bool nan_in) {
#pragma unroll
  for (int j = 0; j < NOUT; ++j) {
    const float4* wa = reinterpret_cast<const float4*>(w3 + 32 * j);
    const float4 va[4] = {wa[0], wa[1], wa[2], wa[3]};
    scr[j * WAVE] = head_dot(va, y0, y1, b3[j], nan_in);
  }
}

// Wide heads (VBN_F_HEAD_MFMA: mdn, softmax_nn; 8..32 outputs) on the split-f16 MFMA like
// layer 2: the layer-2 activations are already in the B-operand layout, W3 is packed as layer
// 2's A fragments (output rows padded to 32) and the bias is the accumulator init, so the head
// is 6 MFMAs and one f16 split per group instead of 16 FMAs per output per group.  Lane half h
// of group g then holds outputs row(r, h) of particle (lane & 31) + 32 g, stored to the head
// rows.  Activations beyond the split range, or a NaN parent input, take the VALU head.
__host__ __device__ constexpr bool head_on_mfma(int flags) {
#ifdef VBN_ABL_NOHEADMFMA      // A/B only: every head on VALU (outputs within an ulp, not bitwise)
  return false;
#else
  return (flags & VBN_F_HEAD_MFMA) != 0 && (flags & VBN_F_F32L2) == 0;
#endif
}

template <int ACT, bool MIR>
__device__ __forceinline__ void head_mfma(const vbn_step& st, const Lane& L, const float* __restrict__ W,
                                          const f32x16& h0, const f32x16& h1, bool nan_in) {
  const int lane = L.lane;
  float y0[16], y1[16];
  int big = 0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    y0[r] = act_fn<ACT>(h0[r]);
    y1[r] = MIR ? y0[r] : act_fn<ACT>(h1[r]);
    big = max(big, max(__float_as_int(y0[r]), __float_as_int(y1[r])));   // positive side only
  }
  if (__any(big > 0x47000000 || nan_in)) {         // rare: the VALU head
    mlp_head<ACT>(st, L, W, h0, h1, nan_in);
    return;
  }
  const float* __restrict__ F = L.P + st.reserved[2];
  const uint4* w3h = reinterpret_cast<const uint4*>(F);
  const uint4 wq[4] = {w3h[lane], w3h[WAVE + lane], w3h[2 * WAVE + lane], w3h[3 * WAVE + lane]};
  const f32x16 bi = load_acc16(F + 1024 + 16 * (lane >> 5));
  const f32x16 o0 = layer2_split(wq, bi, y0);
  const f32x16 o1 = MIR ? o0 : layer2_split(wq, bi, y1);
  const int h = lane >> 5, n = lane & 31;
  float* __restrict__ scr = L.scr;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
    if (row < st.n_out) {
      scr[row * WAVE + n] = o0[r];
      scr[row * WAVE + n + 32] = o1[r];
    }
  }
  wave_sync();
}

// One NN node for the wave's 64 particles from the LDS-staged weight block.  Group 0 (layer 1,
// layer 2 split-f16 on MFMA), group 1, the head on both -- one basic block: the f16 range
// check only ORs a wave-uniform flag, and the rare exact path (an activation beyond the split
// range, or VBN_F_F32L2) re-runs the node on the exact f32 chain after the head and overwrites
// its outputs.  Without branches between them, the compiler can issue group 1's layer-1 /
// split VALU work and group 0's head in the shadow of the other group's MFMAs.  ``pre`` (the
// step's draws) runs after group 0's fragment reads are issued.
template <int ACT, bool STD, int NIN, bool MIR, int NOUT, typename F>
__device__ __forceinline__ void mlp_forward(const vbn_walk_args& A, const vbn_step& st, const Lane& L, F&& pre) {
  const int lane = L.lane;
  const int nin = NIN > 0 ? NIN : st.n_in;
  const float* __restrict__ W = L.wb;
  const uint4* w2h = reinterpret_cast<const uint4*>(W + (OFF_W2H(st) - WBLK_OFF(st)));
  const float* b2 = W + (st.off_b2 - WBLK_OFF(st)) + 64 + 16 * (lane >> 5);
  bool nan_in = false;                            // torch keeps NaN through Linear/act
  for (int d = 0; d < nin; ++d) {
    const float v = L.vals[L.ic[st.in_off + d] * WAVE + lane];
    nan_in |= (v != v);
  }
  f32x16 h0, h1;
  bool beyond;                                    // some layer-1 operand beyond the node's bound
  {
#ifdef VBN_ABL_NOFUSE      // A/B only: relu then the plain split (same outputs to f32 rounding)
    constexpr bool FUSE = false;
#else
    constexpr bool FUSE = ACT == VBN_ACT_RELU;    // relu folded into the f16 split
#endif
    float y[16];
    beyond = mlp_l1_act<ACT, STD, NIN, 0, FUSE>(A, st, L, W, 0, y, pre);
    const uint4 wq[4] = {w2h[lane], w2h[WAVE + lane], w2h[2 * WAVE + lane], w2h[3 * WAVE + lane]};
    h0 = FUSE ? layer2_split_relu(wq, load_acc16(b2), y) : layer2_split(wq, load_acc16(b2), y);
    if constexpr (MIR) {
      h1 = h0;                                    // group 1 = group 0's particles
    } else {
      float y1[16];
      beyond |= mlp_l1_act<ACT, STD, NIN, 0, FUSE>(A, st, L, W, 1, y1, [] {});
      h1 = FUSE ? layer2_split_relu(wq, load_acc16(b2 + 32), y1) : layer2_split(wq, load_acc16(b2 + 32), y1);
    }
  }
  if constexpr (NOUT > 0) {
    float y0[16], y1[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      y0[r] = act_fn<ACT>(h0[r]);
      y1[r] = act_fn<ACT>(h1[r]);
    }
    head_outputs_n<NOUT>(W + (st.off_w3 - WBLK_OFF(st)) + 16 * (lane >> 5), W + (st.off_b3 - WBLK_OFF(st)),
                         L.scr + lane, y0, y1, nan_in);
    wave_sync();
  } else if (head_on_mfma(st.flags)) {
    head_mfma<ACT, MIR>(st, L, W, h0, h1, nan_in);
  } else {
    mlp_head<ACT>(st, L, W, h0, h1, nan_in);
  }
  // rare: an operand beyond the bound -- check the activations themselves (recomputed from the
  // blob: the same values); beyond the split range, the exact f32 chain overwrites the outputs
#ifdef VBN_ABL_NOEXACT   // measurement only: no exact-path branch (wrong when it is needed)
  if (false) {
#else
  if (beyond || (st.flags & VBN_F_F32L2)) {
#endif
    const float* __restrict__ Wg = L.P + WBLK_OFF(st);
    bool big = (st.flags & VBN_F_F32L2) != 0;
    if (!big) {
      float y[16];
      big = mlp_l1_act<ACT, STD, NIN, 1>(A, st, L, Wg, 0, y, [] {});
      if constexpr (!MIR) big |= mlp_l1_act<ACT, STD, NIN, 1>(A, st, L, Wg, 1, y, [] {});
    }
    if (big) {                                    // the exact f32 chain, outputs overwritten
      float y[16];
      mlp_l1_act<ACT, STD, NIN>(A, st, L, Wg, 0, y, [] {});
      h0 = layer2_exact(st, L, 0, y);
      if constexpr (MIR) {
        h1 = h0;
      } else {
        mlp_l1_act<ACT, STD, NIN>(A, st, L, Wg, 1, y, [] {});
        h1 = layer2_exact(st, L, 1, y);
      }
      mlp_head<ACT>(st, L, W, h0, h1, nan_in);
    }
  }
}

// Non-relu activations (kind-set bit 5) take the generic fan-in loop only: a compile-time fan-in
// per activation multiplied the inlined MLP copies of those kind sets by 4 (their objects took
// ~40 min each to build); relu -- the reference default and every benchmark DAG -- keeps them.
template <int ACT, bool STD, bool MIR, int NOUT, typename F>
__device__ __forceinline__ void mlp_nin(const vbn_walk_args& A, const vbn_step& st, const Lane& L, F&& pre) {
  if constexpr (ACT != VBN_ACT_RELU) {
    mlp_forward<ACT, STD, 0, MIR, NOUT>(A, st, L, pre);
  } else {
  switch (st.n_in) {
    case 1: mlp_forward<ACT, STD, 1, MIR, NOUT>(A, st, L, pre); break;
    case 2: mlp_forward<ACT, STD, 2, MIR, NOUT>(A, st, L, pre); break;
    case 3: mlp_forward<ACT, STD, 3, MIR, NOUT>(A, st, L, pre); break;
    default: mlp_forward<ACT, STD, 0, MIR, NOUT>(A, st, L, pre); break;
  }
  }
}

// ------------------------------------------------------------------------------------------
// Generic MLP (any hidden_dims, reference gaussian_nn.py:16-34 _build_mlp; VBN_F_MLP_GENERIC):
// every layer -- input layer, hidden layers, head -- as exact f32 v_mfma_f32_32x32x2_f32 tiles
// of 32 units x 32 particles, K in steps of 2, activations ping-ponged through the wave's LDS
// scratch rows (layer input row k of particle n at buf[k][n]; conflict-free: lane halves read
// rows 2t and 2t + 1).  Out of line so the (32, 32) hot path keeps its registers.
//   off_w2 (step) -> layer table int32 [1 + 4 L]: L, then per layer (in, out, off_w, off_b);
//   off_w : [ceil(out/32)][ceil(in/2)][64]  lane l: W[32 blk + (l & 31)][2 t + (l >> 5)] (0-padded)
//   off_b : [ceil(out/32)][2][16]           b[32 blk + row(r, h)] (accumulator init, 0-padded)
// Scratch rows: [0, n_out) the head's outputs (what the CPD epilogues read), then two buffers
// of max(hidden) rows (plan.py sizes max_out = n_out + 2 max(hidden)).
// ------------------------------------------------------------------------------------------
template <int ACT, bool STD>
__device__ __attribute__((noinline)) void mlp_generic(const vbn_walk_args& A, const vbn_step& st, const Lane& L) {
  const int lane = L.lane, h = lane >> 5, col = lane & 31;
  const cint* tab = CI(L.P + st.off_w2);
  const int nl = tab[0];
  int hmax = 1;
  for (int li = 0; li + 1 < nl; ++li) hmax = max(hmax, tab[2 + 4 * li]);
  float* buf0 = L.scr + st.n_out * WAVE;
  float* buf1 = buf0 + hmax * WAVE;
  bool nan_in = false;                            // torch keeps NaN through Linear / activation
  for (int d = 0; d < st.n_in; ++d) {
    const float v = L.vals[L.ic[st.in_off + d] * WAVE + lane];
    nan_in |= (v != v);
  }
  for (int li = 0; li < nl; ++li) {
    const int in = tab[1 + 4 * li], out = tab[2 + 4 * li];
    const float* __restrict__ W = L.P + tab[3 + 4 * li];
    const float* __restrict__ Bs = L.P + tab[4 + 4 * li];
    const bool last = li + 1 == nl;
    const float* src = (li & 1) ? buf0 : buf1;    // layer li >= 1 reads what li - 1 wrote
    float* dst = last ? L.scr : ((li & 1) ? buf1 : buf0);
    const int nblk = (out + 31) >> 5, t1 = (in + 1) >> 1;
    for (int blk = 0; blk < nblk; ++blk) {
      for (int g = 0; g < 2; ++g) {
        f32x16 a = load_acc16(Bs + blk * 32 + 16 * h);
        for (int t = 0; t < t1; ++t) {
          const float w = W[(blk * t1 + t) * WAVE + lane];
          float x;
          if (li == 0) {
            x = l1_operand<STD, 0>(A, st, L, t, g);
          } else {
            const int k = 2 * t + h;
            x = k < in ? src[k * WAVE + col + 32 * g] : 0.f;
          }
          a = __builtin_amdgcn_mfma_f32_32x32x2f32(w, x, a, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 32 * blk + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (row < out) dst[row * WAVE + col + 32 * g] = last ? a[r] : act_fn<ACT>(a[r]);
        }
      }
    }
    wave_sync();
  }
  if (nan_in)
    for (int j = 0; j < st.n_out; ++j) L.scr[j * WAVE + lane] = __int_as_float(0x7fc00000);
  wave_sync();
}

template <unsigned KM>
__device__ __forceinline__ void run_mlp_generic(const vbn_walk_args& A, const vbn_step& st, const Lane& L) {
  const bool sd = (st.flags & VBN_F_STANDARDIZE) != 0;
  if (!(KM & 32) || st.act == VBN_ACT_RELU) {
    if (sd) mlp_generic<VBN_ACT_RELU, true>(A, st, L); else mlp_generic<VBN_ACT_RELU, false>(A, st, L);
    return;
  }
  if constexpr ((KM & 32) != 0) {
    switch (st.act * 2 + (sd ? 1 : 0)) {
      case 2: mlp_generic<VBN_ACT_TANH, false>(A, st, L); break;
      case 3: mlp_generic<VBN_ACT_TANH, true>(A, st, L); break;
      case 4: mlp_generic<VBN_ACT_GELU, false>(A, st, L); break;
      case 5: mlp_generic<VBN_ACT_GELU, true>(A, st, L); break;
      case 6: mlp_generic<VBN_ACT_ELU, false>(A, st, L); break;
      default: mlp_generic<VBN_ACT_ELU, true>(A, st, L); break;
    }
  }
}

// KM bit 5: some NN CPD uses a non-relu activation; bit 6: half-wave instantiation.  ``pre``:
// the step's draws (see mlp_forward).  NOUT > 0: the caller's head width is a compile-time
// constant (gaussian_nn with D = 1: loc, scale).
template <unsigned KM, int NOUT = 0, typename F>
__device__ __forceinline__ void run_mlp(const vbn_walk_args& A, const vbn_step& st, const Lane& L, F&& pre) {
  constexpr bool MIR = (KM & 64) != 0;             // half-wave instantiation
  if (st.flags & VBN_F_PRECOMP) {                  // parents = shared root draws / evidence: this
    pre();                                         // sample's / query's head outputs, pre-pass
    if (st.flags & VBN_F_PRECOMP_Q) {
      const cfloat* q = precomp_qrow(A, st, L);
      for (int j = 0; j < st.n_out; ++j) L.scr[j * WAVE + L.lane] = q[j];
    } else {
      const float* __restrict__ q = precomp_row(A, st, L);
      for (int j = 0; j < st.n_out; ++j) L.scr[j * WAVE + L.lane] = q[j];
    }
    wave_sync();
    return;
  }
  if constexpr ((KM & 512) != 0) {                 // kind-set bit 9: plans with generic MLPs
    if (st.flags & VBN_F_MLP_GENERIC) {            // hidden_dims other than (32, 32)
      pre();
      run_mlp_generic<KM>(A, st, L);
      return;
    }
  }
  const bool sd = (st.flags & VBN_F_STANDARDIZE) != 0;
  if (!(KM & 32) || st.act == VBN_ACT_RELU) {
    if (sd) mlp_nin<VBN_ACT_RELU, true, MIR, NOUT>(A, st, L, pre);
    else mlp_nin<VBN_ACT_RELU, false, MIR, NOUT>(A, st, L, pre);
    return;
  }
  if constexpr ((KM & 32) != 0) {
    switch (st.act * 2 + (sd ? 1 : 0)) {
      case 2: mlp_nin<VBN_ACT_TANH, false, MIR, NOUT>(A, st, L, pre); break;
      case 3: mlp_nin<VBN_ACT_TANH, true, MIR, NOUT>(A, st, L, pre); break;
      case 4: mlp_nin<VBN_ACT_GELU, false, MIR, NOUT>(A, st, L, pre); break;
      case 5: mlp_nin<VBN_ACT_GELU, true, MIR, NOUT>(A, st, L, pre); break;
      case 6: mlp_nin<VBN_ACT_ELU, false, MIR, NOUT>(A, st, L, pre); break;
      default: mlp_nin<VBN_ACT_ELU, true, MIR, NOUT>(A, st, L, pre); break;
    }
  }
}

// value of node dim d for this particle: fresh draw result or fixed input
#define NODE_X(d) (vread(L, st.out_col + (d)))

// ------------------------------------------------------------------------------------------
// gaussian_nn (gaussian_nn.py:215-288)
//   tail (non-root): std_y[D], mean_y[D], min_scale
//   tail (root)    : loc[D], scale[D], log_scale[D]
// ------------------------------------------------------------------------------------------
template <unsigned KM>
__device__ __forceinline__ void step_gaussian_nn(const vbn_walk_args& A, const vbn_step& st, const Lane& L, float& lp) {
#pragma clang fp contract(off)
  const float* __restrict__ P = L.P;
  const int D = st.out_dim;
  const bool latent = st.role == VBN_ROLE_LATENT;
  const bool want_lp = (st.flags & VBN_F_LOGP) != 0;
  const cfloat* t = CP(P + st.off_tail);
  if (st.flags & VBN_F_ROOT) {
    for (int d = 0; d < D; ++d) {
      const float loc = t[d], scale = t[D + d];
      if (st.role == VBN_ROLE_PARAMS) {
        vwrite(L, st.out_col + d, loc);
        vwrite(L, st.out_col + D + d, scale);
        continue;
      }
      float x;
      if (latent) {
        x = draw_normal(A, st, d, L) * scale + loc;  // torch.normal(loc, scale)
        vwrite(L, st.out_col + d, x);
      } else {
        x = node_fixed(A, st, d, L);
        vwrite(L, st.out_col + d, x);
      }
      if (want_lp) {                                 // Normal.log_prob (gaussian_nn.py:276-279)
        const float diff = x - loc;
        lp += -(diff * diff) / (2.0f * (scale * scale)) - t[2 * D + d] - 0.91893853320467274178f;
      }
    }
    return;
  }
  float eps0 = 0.f;                                 // dim-0 draw, issued beside the weight loads
  auto pre = [&]() { if (latent) eps0 = draw_normal(A, st, 0, L); };
  if (D == 1) run_mlp<KM, 2>(A, st, L, pre);        // head = (loc, raw scale): straight-line
  else run_mlp<KM>(A, st, L, pre);
  const float min_scale = t[2 * D];
  float acc = 0.f;
  for (int d = 0; d < D; ++d) {
    const float o_loc = L.scr[d * WAVE + L.lane];
    const float o_sc = L.scr[(D + d) * WAVE + L.lane];
    const float sy = t[d], my = t[D + d];
    const float loc = o_loc * sy + my;
    const float scale = (softplus_t(o_sc) + min_scale) * sy;
    if (st.role == VBN_ROLE_PARAMS) {
      vwrite(L, st.out_col + d, loc);
      vwrite(L, st.out_col + D + d, scale);
      continue;
    }
    float x;
    if (latent) {
      x = loc + (d == 0 ? eps0 : draw_normal(A, st, d, L)) * scale;
    } else {
      x = node_fixed(A, st, d, L);
    }
    vwrite(L, st.out_col + d, x);
    if (want_lp) {
      const float diff = x - loc;
      acc += (diff * diff) / (scale * scale) + 2.0f * log_hw(scale) + LOG_2PI_F;   // scale >= min_scale std_y
    }
  }
  if (want_lp) lp += -0.5f * acc;
}

// ------------------------------------------------------------------------------------------
// linear_gaussian (linear_gaussian.py:163-217)
//   tail: W[D][n_in] (W[:, d] of the reference's [n_in, D]), bias[D], scale[D], log_scale[D]
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void step_linear_gaussian(const vbn_walk_args& A, const vbn_step& st, const Lane& L, float& lp) {
#pragma clang fp contract(off)
  const float* __restrict__ P = L.P;
  const int D = st.out_dim, nin = st.n_in;
  const cfloat* t = CP(P + st.off_tail);
  const cfloat* W = t;
  const cfloat* bias = t + D * nin;
  const cfloat* scale = bias + D;
  const cfloat* log_scale = scale + D;
  const bool latent = st.role == VBN_ROLE_LATENT;
  float acc = 0.f;
  for (int d = 0; d < D; ++d) {
    float mu = 0.f;
    for (int i = 0; i < nin; ++i) mu = fmaf(vread(L, L.ic[st.in_off + i]), W[d * nin + i], mu);
    const float loc = (nin > 0) ? mu + bias[d] : bias[d];
    if (st.role == VBN_ROLE_PARAMS) {
      vwrite(L, st.out_col + d, loc);
      vwrite(L, st.out_col + D + d, scale[d]);
      continue;
    }
    float x;
    if (latent) {
      x = loc + draw_normal(A, st, d, L) * scale[d];
    } else {
      x = node_fixed(A, st, d, L);
    }
    vwrite(L, st.out_col + d, x);
    if (st.flags & VBN_F_LOGP) {
      const float diff = x - loc;
      acc += (diff * diff) / (scale[d] * scale[d]) + 2.0f * log_scale[d] + LOG_2PI_F;
    }
  }
  if (st.flags & VBN_F_LOGP) lp += -0.5f * acc;
}

// ------------------------------------------------------------------------------------------
// categorical inverse-CDF: smallest k with cumsum(p)[k] > u * sum(p)
// ------------------------------------------------------------------------------------------
// Without an early exit: the first crossing is kept by selects, so a wave whose lanes cross at
// different k runs one straight pass instead of a divergent loop (the divergent form held the
// mdn / softmax_nn epilogues' values live across exec-mask joins: cfg3 spilled 46 VGPRs)
template <typename F>
__device__ __forceinline__ int inv_cdf(int K, float u, F prob) {
  float tot = 0.f;
  for (int k = 0; k < K; ++k) tot += prob(k);
  const float thr = u * tot;
  float cum = 0.f;
  int idx = K - 1;
  bool found = false;
  for (int k = 0; k < K - 1; ++k) {
    cum += prob(k);
    const bool hit = !found && cum > thr;
    idx = hit ? k : idx;
    found |= hit;
  }
  return idx;
}

// ------------------------------------------------------------------------------------------
// mdn (mdn.py:185-272)
//   non-root: scr = [logits K][comp k: loc D, raw_scale D];  tail: min_scale
//   root    : tail = pi[K], log_pi[K], loc[K*D], scale[K*D], log_scale[K*D], var[K*D],
//             softmax(logits)[K] (unclamped, for the PARAMS role)
// ------------------------------------------------------------------------------------------
template <unsigned KM>
__device__ __forceinline__ void step_mdn(const vbn_walk_args& A, const vbn_step& st, const Lane& L, float& lp) {
#pragma clang fp contract(off)
  const float* __restrict__ P = L.P;
  const int D = st.out_dim, K = st.k;
  const cfloat* t = CP(P + st.off_tail);
  const bool root = (st.flags & VBN_F_ROOT) != 0;
  const bool latent = st.role == VBN_ROLE_LATENT;
  const bool want_lp = (st.flags & VBN_F_LOGP) != 0;
  const int lane = L.lane;
  float* scr = L.scr;
  float min_scale = 0.f, lmax = 0.f, lsum = 1.f, psum = 1.f;
  float u0 = 0.f, eps0 = 0.f;                       // component choice + dim-0 normal
  auto draws = [&]() {
    if (latent) {
      u0 = draw_uniforms(A, st, 0, L).x;
      eps0 = draw_normal(A, st, 0, L);
    }
  };
  // pi = softmax(logits).clamp_min(1e-5); pi /= sum (mdn.py:227-228), computed once per
  // particle into the logit rows (the inverse CDF and the log-prob read pi_k repeatedly).
  // The two normalisations multiply by one reciprocal each (within an ulp of the reference's
  // divisions; cfg3 walk -1.8 %); each exp is computed once and kept in its row
  auto make_pi = [&]() {
    lmax = -INFINITY;
    for (int k = 0; k < K; ++k) lmax = fmaxf(lmax, scr[k * WAVE + lane]);
    lsum = 0.f;
    for (int k = 0; k < K; ++k) {
      const float e = __expf(scr[k * WAVE + lane] - lmax);
      scr[k * WAVE + lane] = e;
      lsum += e;
    }
    psum = 0.f;
    const float rl = __builtin_amdgcn_rcpf(lsum);     // lsum >= 1
    for (int k = 0; k < K; ++k) {
      const float p = fmaxf(scr[k * WAVE + lane] * rl, 1e-5f);
      scr[k * WAVE + lane] = p;
      psum += p;
    }
    psum = fmaxf(psum, 1e-12f);
    const float rp = 1.0f / psum;
    for (int k = 0; k < K; ++k) scr[k * WAVE + lane] = scr[k * WAVE + lane] * rp;
  };
  if (root) draws();
  if (!root) run_mlp<KM>(A, st, L, draws);
  if (st.role == VBN_ROLE_PARAMS) {
    // mixture parameters (CPDHandle.conditional, cpd_handle.py:72-88): softmax(logits) [K]
    // (no clamp), loc [K][D], scale [K][D]; root: the host's softmax / loc / scale constants
    if (root) {
      for (int k = 0; k < K; ++k) vwrite(L, st.out_col + k, t[2 * K + 4 * K * D + k]);
      for (int j = 0; j < K * D; ++j) {
        vwrite(L, st.out_col + K + j, t[2 * K + j]);
        vwrite(L, st.out_col + K + K * D + j, t[2 * K + K * D + j]);
      }
      return;
    }
    const float ms = t[0];
    float mx = -INFINITY, se = 0.f;
    for (int k = 0; k < K; ++k) mx = fmaxf(mx, scr[k * WAVE + lane]);
    for (int k = 0; k < K; ++k) se += __expf(scr[k * WAVE + lane] - mx);
    for (int k = 0; k < K; ++k) vwrite(L, st.out_col + k, __expf(scr[k * WAVE + lane] - mx) / se);
    for (int k = 0; k < K; ++k)
      for (int d = 0; d < D; ++d) {
        vwrite(L, st.out_col + K + k * D + d, scr[(K + k * 2 * D + d) * WAVE + lane]);
        vwrite(L, st.out_col + K + K * D + k * D + d,
               softplus_t(scr[(K + k * 2 * D + D + d) * WAVE + lane]) + ms);
      }
    return;
  }
  if (!root) {
    min_scale = t[0];
    make_pi();
  }
  auto pi_k = [&](int k) -> float { return root ? t[k] : scr[k * WAVE + lane]; };
  auto loc_kd = [&](int k, int d) -> float {
    return root ? t[2 * K + k * D + d] : scr[(K + k * 2 * D + d) * WAVE + lane];
  };
  auto scale_kd = [&](int k, int d) -> float {
    return root ? t[2 * K + K * D + k * D + d]
                : softplus_t(scr[(K + k * 2 * D + D + d) * WAVE + lane]) + min_scale;
  };
  if (latent) {
    const int idx = inv_cdf(K, u0, pi_k);
    for (int d = 0; d < D; ++d)
      vwrite(L, st.out_col + d, loc_kd(idx, d) + (d == 0 ? eps0 : draw_normal(A, st, d, L)) * scale_kd(idx, d));
  } else {
    for (int d = 0; d < D; ++d) vwrite(L, st.out_col + d, node_fixed(A, st, d, L));
  }
  if (want_lp) {
    // logsumexp_k(log pi_k + log N_k(x))  (mdn.py:263-272), online form
    float m = -INFINITY, se = 0.f;
    for (int k = 0; k < K; ++k) {
      float acc = 0.f;
      for (int d = 0; d < D; ++d) {
        const float x = NODE_X(d);
        float ls, var;
        if (root) {
          ls = t[2 * K + 2 * K * D + k * D + d];
          var = t[2 * K + 3 * K * D + k * D + d];
        } else {
          ls = log_hw(scale_kd(k, d));                 // scale >= min_scale
          var = __expf(2.0f * ls);
        }
        const float diff = x - loc_kd(k, d);
        acc += (diff * diff) / var + 2.0f * ls + LOG_2PI_F;
      }
      const float lpi = root ? t[K + k] : log_hw(pi_k(k));   // pi >= 1e-5 / sum
      const float term = lpi + (-0.5f * acc);
      if (term == -INFINITY) continue;
      if (term > m) {
        se = se * __expf(m - term) + 1.0f;
        m = term;
      } else {
        se += __expf(term - m);
      }
    }
    lp += (m == -INFINITY) ? m : m + log_hw(se);          // se >= 1
  }
}

// ------------------------------------------------------------------------------------------
// softmax_nn (softmax_nn.py:581-759)
//   scr (non-root) = logits[D][C];  root logits table at off_pts ([D][C], already log_softmax'd)
//   tail: edges[D][C+1], sample_values[D][C], class_values[D][C], within_scale, min_bw, min_bw2
//   aux0 = within-bin mode, aux1 = discrete-dim bit mask
// ------------------------------------------------------------------------------------------
template <unsigned KM>
__device__ __forceinline__ void step_softmax_nn(const vbn_walk_args& A, const vbn_step& st, const Lane& L, float& lp) {
#pragma clang fp contract(off)
  const float* __restrict__ P = L.P;
  const int D = st.out_dim, C = st.k;
  const cfloat* t = CP(P + st.off_tail);
  const cfloat* edges = t;
  const cfloat* svals = t + D * (C + 1);
  const cfloat* cvals = svals + D * C;
  const float wscale = cvals[D * C + 0];
  const float min_bw = cvals[D * C + 1];
  const float min_bw2 = cvals[D * C + 2];
  const bool root = (st.flags & VBN_F_ROOT) != 0;
  const bool latent = st.role == VBN_ROLE_LATENT;
  const bool clip = (st.flags & VBN_F_CLIP) != 0;
  const int mode = st.aux0;
  const int lane = L.lane;
  float2 uu0 = make_float2(0.f, 0.f);               // dim-0 uniforms
  auto draws = [&]() { if (latent) uu0 = draw_uniforms(A, st, 0, L); };
  if (root) draws(); else run_mlp<KM>(A, st, L, draws);
  float lp_acc = 0.f;
  for (int d = 0; d < D; ++d) {
    auto logit = [&](int c) -> float {
      return root ? P[st.off_pts + d * C + c] : L.scr[(d * C + c) * WAVE + lane];
    };
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = fmaxf(m, logit(c));
    float se = 0.f;
    // a latent non-root step without a log-prob reads the logits only here: each exp is
    // computed once and kept in its row for the class probabilities below (same values)
    const bool keep_e = latent && !root && !(st.flags & VBN_F_LOGP);
    if (keep_e) {
      for (int c = 0; c < C; ++c) {
        const float e = __expf(logit(c) - m);
        L.scr[(d * C + c) * WAVE + lane] = e;
        se += e;
      }
    } else {
      for (int c = 0; c < C; ++c) se += __expf(logit(c) - m);
    }
    if (st.role == VBN_ROLE_PARAMS) {   // softmax(logits) per dim: [D][C] (RB target: D = 1)
      for (int c = 0; c < C; ++c) vwrite(L, st.out_col + d * C + c, __expf(logit(c) - m) / se);
      continue;
    }
    const bool disc = (st.aux1 >> d) & 1;
    const cfloat* e = edges + d * (C + 1);
    float x;
    int idx;
    if (latent) {
      const float2 uu = d == 0 ? uu0 : draw_uniforms(A, st, d, L);
      if (keep_e) {
        // the logits are not read again: the class probabilities replace the kept exps
        // (the inverse CDF reads each twice; same operations, so the same values); one
        // reciprocal of the sum instead of C divisions
        const float rse = __builtin_amdgcn_rcpf(se);  // se >= 1
        for (int c = 0; c < C; ++c) L.scr[(d * C + c) * WAVE + lane] = L.scr[(d * C + c) * WAVE + lane] * rse;
        idx = inv_cdf(C, uu.x, [&](int c) { return L.scr[(d * C + c) * WAVE + lane]; });
      } else {
        const float rse = __builtin_amdgcn_rcpf(se);  // se >= 1
        idx = inv_cdf(C, uu.x, [&](int c) { return __expf(logit(c) - m) * rse; });
      }
      const float left = e[idx];
      const float right = e[idx + 1 < C ? idx + 1 : C];
      const float width = fmaxf(right - left, min_bw);
      const float center = 0.5f * (left + right);
      if (disc) {
        x = svals[d * C + idx];
      } else {
        float cont;
        if (mode == VBN_WITHIN_UNIFORM) {
          cont = left + uu.y * width;
        } else if (mode == VBN_WITHIN_TRIANGULAR) {
          // only the chosen side's root (the same operations on the same values)
          const bool lo = uu.y < 0.5f;
          const float r = sqrtf(fmaxf((lo ? uu.y : 1.0f - uu.y) * 0.5f, 0.0f));
          cont = lo ? left + width * r : right - width * r;
        } else {
          cont = center + draw_normal(A, st, d, L) * fmaxf(wscale * width, min_bw);
        }
        if (clip) cont = fminf(fmaxf(cont, left), right);
        x = cont;
      }
    } else {
      x = node_fixed(A, st, d, L);
    }
    vwrite(L, st.out_col + d, x);
    if (st.flags & VBN_F_LOGP) {
      // bin: count(x >= edges) - 1 clamped (bit-exact); discrete: first exact class match
      int bin;
      if (disc) {
        bin = 0;
        for (int c = C - 1; c >= 0; --c)
          if (x == cvals[d * C + c]) bin = c;
      } else {
        int cnt = 0;
        for (int c = 0; c <= C; ++c) cnt += (x >= e[c]) ? 1 : 0;
        bin = min(max(cnt - 1, 0), C - 1);
      }
      const float log_bin = logit(bin) - m - log_hw(se);
      float lw = 0.f;
      if (!disc) {
        const float left = e[bin];
        const float right = e[bin + 1 < C ? bin + 1 : C];
        const float width = fmaxf(right - left, min_bw);
        const float center = 0.5f * (left + right);
        const float xu = clip ? fminf(fmaxf(x, left), right) : x;
        const bool inside = (x >= left) && (x <= right);
        if (mode == VBN_WITHIN_UNIFORM) {
          lw = -log_hw(width);
          if (!clip && !inside) lw = -INFINITY;
        } else if (mode == VBN_WITHIN_TRIANGULAR) {
          const float dl = fmaxf(width * (center - left), min_bw2);
          const float dr = fmaxf(width * (right - center), min_bw2);
          float pdf = (xu <= center) ? 2.0f * (xu - left) / dl : 2.0f * (right - xu) / dr;
          pdf = fmaxf(pdf, 0.0f);
          lw = log_hw(fmaxf(pdf, 1e-12f));
          if (!clip && !inside) lw = -INFINITY;
        } else {
          const float sigma = fmaxf(wscale * width, min_bw);
          const float diff = xu - center;
          lw = -(diff * diff) / (2.0f * (sigma * sigma)) - log_hw(sigma) - 0.91893853320467274178f;
        }
      }
      lp_acc += log_bin + lw;
    }
  }
  if (st.flags & VBN_F_LOGP) lp += lp_acc;
}

// ------------------------------------------------------------------------------------------
// kde (kde.py:105-182)
//   points at off_pts: [M][stride] = parents[dp] ++ targets[D]
//   tail: inv_sp, inv_sy, noise_scale, cy, log_n;  aux0 = dp, aux1 = stride
// Weights are taken relative to the kernel's peak (exp(-q/2) <= 1); if every weight of a
// particle underflows the pass is redone relative to the particle's nearest point.
// ------------------------------------------------------------------------------------------
// squared scaled distance to point ``pt`` over the parent dims.  DP >= 0: parent values in
// registers (pv); DP < 0: generic count, parent values re-read from LDS.
template <int DP>
__device__ __forceinline__ float kde_qp(const float* __restrict__ pt, const float (&pv)[4], float inv,
                                        int dp, const vbn_walk_args& A, const vbn_step& st, const Lane& L) {
  float q = 0.f;
  if (DP >= 0) {
#pragma unroll
    for (int i = 0; i < (DP >= 0 ? DP : 0); ++i) {
      const float df = (pv[i] - pt[i]) * inv;
      q = fmaf(df, df, q);
    }
  } else {
    for (int i = 0; i < dp; ++i) {
      const float df = (vread(L, L.ic[st.in_off + i]) - pt[i]) * inv;
      q = fmaf(df, df, q);
    }
  }
  return q;
}

template <int DY>
__device__ __forceinline__ float kde_qy(const float* __restrict__ pty, float x0, float inv, int D,
                                        const vbn_step& st, const Lane& L) {
  if (DY == 1) {
    const float df = (x0 - pty[0]) * inv;
    return df * df;
  }
  float q = 0.f;
  for (int d = 0; d < D; ++d) {
    const float df = (vread(L, st.out_col + d) - pty[d]) * inv;
    q = fmaf(df, df, q);
  }
  return q;
}

// ---- pairwise kernel weights on MFMA ------------------------------------------------------
// The kernel weight of particle n and stored point m is exp(-|x_n - y_m|^2 / (2 s^2)) =
// exp2(-|x'_n - y'_m|^2) with x' = c x, y' = c y, c = sqrt(log2(e) / 2) / s, and
//   -|x' - y'|^2 = sum_k (2 x'_k) y'_k - |y'|^2 - |x'|^2,
// a contraction over K <= 4 features, computed on bf16 MFMAs from exact three-way splits
// (kde_b32_sums below) for the inverse-CDF chunk sums and the log-density sums alike.
// Padding points have |y'|^2 = 1e30 -> weight 0.  The wave's 64 particles are 2 tiles of 32
// (tile t = particles 32t .. 32t+31); D layout: lane l holds points 8j + 4(l>>5) + i (j, i < 4)
// of the block for particle 32t + (l&31).  Bound: v_exp_f32 issue (one exp per pair).  The inverse-CDF scan
// recomputes its chunk's weights with kde_arg_rec, the float32 chain of the same contraction
// (equal to the MFMA sums to f32 rounding; a crossing past the chunk end is clamped, kde_scan).
// the lane's own particle: x'_k and -|x'|^2 exactly as kde_b32_ops computes them
__device__ __forceinline__ float kde_own(const Lane& L, const int (&slots)[4], const float (&scl)[4], int nf,
                                         float (&xv)[4]) {
  float sq = 0.f;
  for (int f = 0; f < nf; ++f) {
    const float v = scl[f] * vread(L, slots[f]);
    xv[f] = v;
    sq = fmaf(v, v, sq);
  }
  return -sq;
}

// VALU form of one pair's argument (a k-ordered fmaf chain), point record r =
// (y'_0 .. y'_{nf-1}, |y'|^2, ..) of the per-point record pack.
__device__ __forceinline__ float kde_arg_rec(const float4 r, float xb0, float xb1, float xb2, float negsq,
                                             int nf) {
  const bool zc = nf <= 2;
  float d = zc ? 0.f : negsq;
  d = fmaf(r.x, xb0, d);
  d = nf > 1 ? fmaf(r.y, xb1, d) : d;
  d = nf > 2 ? fmaf(r.z, xb2, d) : d;
  const float y2 = nf == 1 ? r.y : (nf == 2 ? r.z : r.w);
  d = fmaf(y2, -1.f, d);
  return zc ? fmaf(1.f, negsq, d) : d;
}

// 16-point blocks per chunk: a multiple of 4, so a chunk is a whole number of the MFMA pass's
// KDE_PF = 2 blocks of 32 points (the host pads the packs to KDE_CHUNKS * kde_cb(M) 16-point
// blocks)
__device__ __forceinline__ int kde_cb(int M) {
  const int nblk = (M + 15) >> 4;
  return (((nblk + KDE_CHUNKS - 1) / KDE_CHUNKS) + 3) & ~3;
}

// Point operands are prefetched a whole trip ahead, across chunk boundaries: the packs of a
// 64-node M = 10,000 DAG do not stay in one XCD's 4 MiB L2 while ~4,000 resident waves walk
// different nodes, so most operand loads are served by the Infinity Cache (cfg4: 78 GB of L2
// fills per launch, r04 PMC), ~545+ cycles away.  Measured not to cost time: re-reading only
// the first 32 blocks of every pack (VBN_ABL_L2FIT, L2-resident) ran 202.5 vs 201.0 ms.

#ifdef VBN_ABL_L2FIT
#define KDE_BLK(x) ((x) & 31)        // ablation: every pass re-reads its node's first 32 blocks
#else
#define KDE_BLK(x) (x)
#endif

// Pass-1 sums on v_mfma_f32_32x32x16_bf16 ("bf16x3", round 5): rows = 32 points, columns =
// the 32 particles of tile t (particles 32 t .. 32 t + 31), K = 16 slots (one MFMA, nf = 1) or
// 32 (two chained MFMAs, nf = 2..4).  Every f32 operand is split into three bf16 whose sum is
// it exactly (hi = bf16(v), mid = bf16(v - hi), lo = the 8-bit rest); per feature f the six
// products u_h y_h, u_h y_m, u_m y_h, u_h y_l, u_l y_h, u_m y_m (u = 2x' on the B side, y' on
// the A side, slots 6f .. 6f+5; the omitted ones are < 2^-25 of u y) are exact in f32,
// |y'|^2's three parts (slots 6nf .. +2) meet -1 and 1.0 (6nf+3 .. +5) meets -|x'|^2's three
// parts, so the MFMA's f32 sum from C = 0 is the contraction -|x' - y'|^2 to f32 rounding
// (tests/test_plan.py).  Against round 4's v_mfma_f32_16x16x32_bf16 tiles the wave issues a
// quarter of the MFMAs per pair (one 32x32x16 per 1,024 pairs instead of four 16x16x32, each
// holding the SIMD's vector issue for 8 cycles) and reads 32 instead of 64 bytes per point
// for nf = 1; the 16 exps per lane and MFMA are summed with plain f32 adds (4 accumulators
// per tile; packed f32 adds beside MFMAs cost extra issue cycles, MI355X_MICROARCH.md).
// A = host pack (plan.py _kde_pack_b32) [block of 32][K group g][64 lanes][8]: lane l loads
// point l & 31's slots 16 g + 8 (l >> 5) .. +7 (16 B, 1 KiB per wave, block and K group);
// B = kde_b32_ops; D: lane l holds rows 8 j + 4 (l >> 5) + i (j, i < 4) of column l & 31.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int KG>
struct KdeB32 {
  bf16x8 b[2][KG];  // tile t: particle 32 t + (lane & 31), slots 16 g + 8 (lane >> 5) .. +7
};

__device__ __forceinline__ void bf16_split3(float v, __bf16 (&p)[3]) {
  p[0] = (__bf16)v;
  const float r1 = v - (float)p[0];
  p[1] = (__bf16)r1;
  p[2] = (__bf16)(r1 - (float)p[1]);
}

// slot k of the B operand: feature splits sp (_BF16_B pattern), -1 x 3, split of -|x'|^2 (zero
// in the factored form: the A side's 1.0 slots then contribute nothing), 0
__device__ __forceinline__ __bf16 kde_bslot(int k, int nf, const __bf16 (&sp)[4][3], const __bf16 (&sx)[3],
                                            bool fform) {
  constexpr int pat[6] = {0, 0, 1, 0, 2, 1};
  const int f = k / 6;
  if (f < nf) return sp[f][pat[k - 6 * f]];
  const int r = k - 6 * nf;
  if (r < 3) return (__bf16)-1.f;
  if (r < 6 && !fform) return sx[r - 3];
  return (__bf16)0.f;
}

// the lane's particle side of tile t; -|x'|^2 exactly as kde_own accumulates it
template <int KG>
__device__ __forceinline__ void kde_b32_ops(const Lane& L, const int (&slots)[4], const float (&scl)[4], int nf,
                                            bool fform, KdeB32<KG>& o) {
  const int h = L.lane >> 5, n = L.lane & 31;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float sq = 0.f;
    __bf16 sp[4][3], sx[3];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const float v = f < nf ? scl[f] * L.vals[slots[f] * WAVE + 32 * t + n] : 0.f;
      if (f < nf) sq = fmaf(v, v, sq);
      bf16_split3(2.f * v, sp[f]);
    }
    bf16_split3(-sq, sx);
#pragma unroll
    for (int g = 0; g < KG; ++g) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const __bf16 v0 = kde_bslot(16 * g + j, nf, sp, sx, fform);
        const __bf16 v1 = kde_bslot(16 * g + 8 + j, nf, sp, sx, fform);
        o.b[t][g][j] = h ? v1 : v0;
      }
    }
  }
}

// Sum over a chunk's 32-point blocks of the lane's tile partials: lane l receives the total of
// particle l (tile l >> 5, column l & 31): one cross-lane move.
__device__ __forceinline__ float kde_reduce_tiles(const float (&s)[2], int lane) {
  const int h = lane >> 5;
  const float k = h ? s[1] : s[0], o = h ? s[0] : s[1];
  return k + __shfl_xor(o, 32);
}

// One tile of one 32-point block: KG chained MFMAs (C = 0)
template <int KG>
__device__ __forceinline__ f32x16 kde_b32_tile(const bf16x8 (&a)[KG], const bf16x8 (&b)[KG]) {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  f32x16 d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], z, 0, 0, 0);
  if constexpr (KG == 2) d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], d, 0, 0, 0);
  return d;
}

// A tile's 16 exps summed into its 4 accumulators (in the order i = 0 .. 15, so the same sums
// whatever the MFMA schedule)
template <int KG>
__device__ __forceinline__ void kde_b32_exps(const f32x16& d, float (&acc)[4]) {
  if constexpr (KG == 1) {
    // f32x2 adds, one v_pk_add_f32 per two exps: 0.69 vs 0.63 of the exp-issue peak with
    // plain adds (profiles/microbench/kde_pass1.hip w1p / w1s); beside the denser chained
    // MFMAs of K = 32 they gain nothing (w2u 0.600 vs w2t 0.597), so that form keeps plain adds
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
      f32x2 p0 = f32x2{acc[0], acc[1]}, p1 = f32x2{acc[2], acc[3]};
      p0 += f32x2{__builtin_amdgcn_exp2f(d[i]), __builtin_amdgcn_exp2f(d[i + 1])};
      p1 += f32x2{__builtin_amdgcn_exp2f(d[i + 2]), __builtin_amdgcn_exp2f(d[i + 3])};
      acc[0] = p0.x; acc[1] = p0.y; acc[2] = p1.x; acc[3] = p1.y;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i & 3] += __builtin_amdgcn_exp2f(d[i]);
  }
}

// block b's operands (clamped to the pack's last block; pa = pack + lane; PG = the pack's K
// groups per block: the factored form of two features reads group 0 of a K = 32 pack)
template <int KG, int PG>
__device__ __forceinline__ void kde_b32_load(const bf16x8* __restrict__ pa, int b, int blast, bf16x8 (&a)[KG]) {
  const int bb = KDE_BLK(min(b, blast));
#pragma unroll
  for (int g = 0; g < KG; ++g) a[g] = pa[(bb * PG + g) * 64];
}

// In flight across a node's blocks (and its chunks): the operands of the next KDE_PF blocks
// (a ring: block b's set is reloaded with block b + KDE_PF once its last MFMA is issued) and
// the tile-0 result of the next block.  The walk is tile-pipelined: tile i + 1's MFMAs are
// issued before tile i's exps, so no exp waits on its MFMA (microbenchmark w1u 0.707 vs w1p
// 0.690, w2t 0.597 vs w2s 0.588 of the exp-issue peak), with two tile results live as before.
#define KDE_PF 2             // kde_cb keeps every chunk a multiple of 2 blocks of 32 points
template <int KG>
struct KdeTrip {
  bf16x8 x[KDE_PF][KG];
  f32x16 d0;                 // tile 0 of the next block
};

template <int KG, int PG>
__device__ __forceinline__ void kde_b32_prefetch(const bf16x8* __restrict__ pa, int b0, int blast,
                                                 const KdeB32<KG>& o, KdeTrip<KG>& q) {
#pragma unroll
  for (int u = 0; u < KDE_PF; ++u) kde_b32_load<KG, PG>(pa, b0 + u, blast, q.x[u]);
  q.d0 = kde_b32_tile<KG>(q.x[0], o.b[0]);
}

// per-lane tile partial sums of exp2(arg) over 32-point blocks [b0, b1), b1 - b0 a multiple of
// KDE_PF (kde_cb); q holds block b0's tile 0 and the operands of blocks b0, b0 + 1
template <int KG, int PG>
__device__ __forceinline__ void kde_b32_sums(const bf16x8* __restrict__ pa, int b0, int b1, int blast,
                                             const KdeB32<KG>& o, float (&s)[2], KdeTrip<KG>& q) {
  float acc[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[t][i] = 0.f;
  for (int b = b0; b < b1; b += KDE_PF) {
#pragma unroll
    for (int u = 0; u < KDE_PF; ++u) {
      const f32x16 d1 = kde_b32_tile<KG>(q.x[u], o.b[1]);              // block b + u, tile 1
      kde_b32_load<KG, PG>(pa, b + u + KDE_PF, blast, q.x[u]);
      kde_b32_exps<KG>(q.d0, acc[0]);                                   // block b + u, tile 0
      q.d0 = kde_b32_tile<KG>(q.x[(u + 1) % KDE_PF], o.b[0]);           // block b + u + 1, tile 0
      kde_b32_exps<KG>(d1, acc[1]);
    }
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) s[t] += (acc[t][0] + acc[t][1]) + (acc[t][2] + acc[t][3]);
}

// The factored form (round 5).  Sampling needs the chunk sums only up to a per-particle
// factor, so they may be taken of exp2(2 x'.y' - |y'|^2) = 2^{|x'|^2} exp2(-|x' - y'|^2): the
// contraction drops -|x'|^2's three slots and fits K = 16 for two features (6 nf + 3 = 15)
// -- one MFMA per block instead of two chained ones, and the f32x2 adds (w1p, 0.69 vs w2s
// 0.59 of the exp-issue peak).  The particle's sums are then shifted by s = -|x'|^2 relative to
// the full form, and the record scan, the all-underflow rescue and the per-sample / per-query
// pre-passes all work on a' = 2 x'.y' - |y'|^2 minus a shift sigma (0 here, |x'|^2 in the full
// form, the largest a' after a rescue).  Used when every lane of the wave has |x'|^2 <=
// KDE_FFORM_MAX (no overflow: sums <= M 2^{|x'|^2}); otherwise the full form.
#define KDE_FFORM_MAX 96.f

// Sub-chunks (round 6; VBN_ABL_NOHALVES: A/B without).  A wave's scan lasts as long as its
// slowest lane's, about half a chunk (the max over 64 lanes of the bidirectional walk).  Pass 1
// therefore also keeps KDE_NSUB - 1 prefix sums per chunk (a private array: the LDS rows are
// the occupancy budget -- 32 chunk rows instead cost 16 -> 12 waves per CU and ran slower), at
// block boundaries kde_sub_blocks(cb32, k) (multiples of KDE_PF, about k / KDE_NSUB of the
// chunk), and the scan covers the sub-chunk holding the threshold.  cfg4 plain plan, one box
// (profiles/r06_bench/r06i_ab_sub.txt): 88.86 ms -> 81.82 (halves) / 81.87 (quarters).
#ifndef KDE_NSUB
#define KDE_NSUB 2
#endif
#define KDE_HALF_MIN 16      // 32-point blocks per chunk below which a chunk is scanned whole
__device__ __forceinline__ int kde_sub_blocks(int cb32, int k) {
  return ((cb32 * k) / KDE_NSUB) & ~(KDE_PF - 1);
}

// Pass 1 of a node with nf features over its KDE_CHUNKS chunks: chunk sums -> scr[chunk][lane]
template <int KG, int PG>
__device__ __forceinline__ double kde_pass1(const bf16x8* __restrict__ pa, int cb32, const Lane& L,
                                            const int (&slots)[4], const float (&scl)[4], int nf, bool fform,
                                            float* __restrict__ hs = nullptr) {
  KdeB32<KG> o;
  kde_b32_ops<KG>(L, slots, scl, nf, fform, o);
  const int blast = KDE_CHUNKS * cb32 - 1;
  KdeTrip<KG> q;
  kde_b32_prefetch<KG, PG>(pa, 0, blast, o, q);
  double tot = 0.0;
  for (int ch = 0; ch < KDE_CHUNKS; ++ch) {
    float s[2] = {0.f, 0.f};
    if (hs) {                                         // the sub-chunk prefix sums on the way
      int b = ch * cb32;
#pragma unroll
      for (int k = 1; k < KDE_NSUB; ++k) {
        const int bk = ch * cb32 + kde_sub_blocks(cb32, k);
        kde_b32_sums<KG, PG>(pa, b, bk, blast, o, s, q);
        hs[ch * (KDE_NSUB - 1) + k - 1] = kde_reduce_tiles(s, L.lane);
        b = bk;
      }
      kde_b32_sums<KG, PG>(pa, b, ch * cb32 + cb32, blast, o, s, q);
    } else {
      kde_b32_sums<KG, PG>(pa, ch * cb32, ch * cb32 + cb32, blast, o, s, q);
    }
    const float cs = kde_reduce_tiles(s, L.lane);
    L.scr[ch * WAVE + L.lane] = cs;
    tot += (double)cs;
  }
  return tot;
}

// Sum over all nb32 blocks of a log-density pack (kde_logp_mfma)
template <int KG, int PG>
__device__ __forceinline__ float kde_sum_all(const bf16x8* __restrict__ pa, int nb32, const Lane& L,
                                             const int (&slots)[4], const float (&scl)[4], int nf, bool fform) {
  KdeB32<KG> o;
  kde_b32_ops<KG>(L, slots, scl, nf, fform, o);
  KdeTrip<KG> q;
  kde_b32_prefetch<KG, PG>(pa, 0, nb32 - 1, o, q);
  float s[2] = {0.f, 0.f};
  kde_b32_sums<KG, PG>(pa, 0, nb32, nb32 - 1, o, s, q);
  return kde_reduce_tiles(s, L.lane);
}

// the form of a pack of nf features: K groups read (KG), K groups per block of the pack (PG)
__device__ __forceinline__ float kde_sums_nf(const bf16x8* __restrict__ pa, int nb32, const Lane& L,
                                             const int (&slots)[4], const float (&scl)[4], int nf, bool fform) {
  if (nf == 1) return kde_sum_all<1, 1>(pa, nb32, L, slots, scl, nf, fform);
  if (nf == 2 && fform) return kde_sum_all<1, 2>(pa, nb32, L, slots, scl, nf, fform);
  return kde_sum_all<2, 2>(pa, nb32, L, slots, scl, nf, fform);
}

// Inverse-CDF scan of one chunk [j0, j1) (pass 2).  A lane whose threshold lies in the upper
// half of its chunk scans backwards from the end for the right-hand mass csum - rem: the
// point found is the same (the largest j with cum(j-1) <= rem), and no lane scans more than
// about half a chunk.  Backward lanes walk the reversed record copy forward, so every lane
// reads 4 consecutive records per trip with the next trip's 4 in flight (two named record sets,
// no register rotation) and no per-lane selects.  The weights exp2(arg(r)) (arg includes the
// shift) are summed in scan order (bit-identical running sums to a point-by-point scan); one
// compare per trip -- c > lim, with lim the float below the goal for backward lanes (c >= goal)
// -- and the crossing inside the trip is located after the loop; a crossing past the chunk end
// (rounding) is clamped to the chunk's last point.  rec: records (plan.py _kde_pack
// records=True), rev = reversed copy; M points.  Against round 4's form (selects inside the
// trip, a register rotation of the next records, the shift as a separate subtraction): cfg4
// plan kernel without precompute 143 -> 137 ms; trips of 8 records lost (145 ms,
// profiles/r05_bench/r05d_ab_scan.txt).
// the largest float below x (x finite): the backward scan's c >= goal as c > float_below(goal)
__device__ __forceinline__ float float_below(float x) {
  const int i = __float_as_int(x);
  return x > 0.f ? __int_as_float(i - 1) : (x == 0.f ? -__int_as_float(1) : __int_as_float(i + 1));
}

template <class ARG>
__device__ __forceinline__ int kde_scan(const float4* __restrict__ rec, const float4* __restrict__ rev, int M,
                                        int j0, int j1, float rem, float csum, ARG arg) {
  const bool back = rem > 0.5f * csum;
  const float goal = back ? csum - rem : rem;
  const float lim = back ? float_below(goal) : goal;
  const float4* __restrict__ q = back ? rev + (M - j1) : rec + j0;
  const int n = j1 - j0;
  float cs = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
  int kt = n;                                   // first point of the crossing trip (n: none)
  float4 a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
  float4 b0 = q[4], b1 = q[5], b2 = q[6], b3 = q[7];
  for (int k = 0; k < n; k += 8) {
    {
      const float e0 = cs + __builtin_amdgcn_exp2f(arg(a0));
      const float e1 = e0 + __builtin_amdgcn_exp2f(arg(a1));
      const float e2 = e1 + __builtin_amdgcn_exp2f(arg(a2));
      const float e3 = e2 + __builtin_amdgcn_exp2f(arg(a3));
      if (e3 > lim) { c0 = e0; c1 = e1; c2 = e2; c3 = e3; kt = k; break; }
      cs = e3;
    }
    a0 = q[k + 8]; a1 = q[k + 9]; a2 = q[k + 10]; a3 = q[k + 11];
    if (k + 4 >= n) break;
    {
      const float e0 = cs + __builtin_amdgcn_exp2f(arg(b0));
      const float e1 = e0 + __builtin_amdgcn_exp2f(arg(b1));
      const float e2 = e1 + __builtin_amdgcn_exp2f(arg(b2));
      const float e3 = e2 + __builtin_amdgcn_exp2f(arg(b3));
      if (e3 > lim) { c0 = e0; c1 = e1; c2 = e2; c3 = e3; kt = k + 4; break; }
      cs = e3;
    }
    b0 = q[k + 12]; b1 = q[k + 13]; b2 = q[k + 14]; b3 = q[k + 15];
  }
  (void)c3;
  const int v = c0 > lim ? 0 : (c1 > lim ? 1 : (c2 > lim ? 2 : 3));
  const int kh = kt < n ? min(kt + v, n - 1) : n - 1;
  return min(max(back ? j1 - 1 - kh : j0 + kh, 0), M - 1);
}

// One-feature node with a moment table (plan.kde_moment_table, round 6): the index of
// kde.py:172-178 without pass 1's exps.  Around the grid centre u_g nearest u = 2 x', a chunk's
// sum is S_c(u) = sum_k d^k T[g][c][k] with d = u - u_g and
// T[g][c][k] = sum_{j in c} exp2(u_g y'_j - |y'_j|^2) (ln2 y'_j)^k / k! (float64 sums, host);
// the series' remainder is < 3e-8 of every weight (plan.KDE_MT_Z), so the sums equal the
// exp-by-exp ones to f32 rounding, at one 16-byte load and 3 FMAs per chunk.  Per cell the
// table holds the chunks (~M/64 points each), their groups of 8 and the whole point set: the
// threshold u * total, then the group whose running sum passes it, then the chunk inside it
// (<= 8 + 8 sums instead of 64), so the scan that follows covers about M/128 points instead of
// the MFMA pass's M/32; a crossing past the last group or chunk (rounding) takes the last.
// Factored form (shift 0): the caller takes this path only when every lane has fform.  Returns
// -1 for the whole wave when some lane's u is off the grid (or NaN): the MFMA pass then runs.
// Table: header [u_lo, 1 / delta, delta, n_cells, n_chunks, chunk points (int32 bits), 0, 0],
// rows [n_cells][n_chunks + n_groups + 1] float4 (plan.kde_moment_table).
#define KDE_MT_HEAD 8         // header floats (plan.KDE_MT_HEADER)
#define KDE_MT_GROUP 8        // chunks per group (plan.KDE_MT_GROUP)
__device__ __forceinline__ int kde_index_moments(const float* __restrict__ T, float xb0, float ucat,
                                                 const float4* __restrict__ rec, int M, float& total) {
  const cfloat* H = CP(T);
  const float u_lo = H[0], inv_d = H[1], dlt = H[2];
  const int n_cells = __float_as_int(H[3]), nch = __float_as_int(H[4]), per = __float_as_int(H[5]);
  const float gr = rintf((xb0 - u_lo) * inv_d);          // nearest centre (NaN u: not in range)
  const bool in = gr >= 0.f && gr < (float)n_cells;
  if (!__all(in)) return -1;
  const float d = xb0 - fmaf(gr, dlt, u_lo);             // the centre exactly as the host formed it
  const int ng = (nch + KDE_MT_GROUP - 1) / KDE_MT_GROUP;
  const float4* __restrict__ row = reinterpret_cast<const float4*>(T + KDE_MT_HEAD) + (int)gr * (nch + ng + 1);
  auto poly = [&](const float4 c) { return fmaf(fmaf(fmaf(c.w, d, c.z), d, c.y), d, c.x); };
  total = poly(row[nch + ng]);
  const double thr = (double)ucat * (double)total;
  double cum = 0.0;
  float gs = 0.f;
  int g = ng - 1;
  bool hit = false;
  for (int k = 0; k < ng; ++k) {                        // the group
    gs = poly(row[nch + k]);
    const double nx = cum + (double)gs;
    if (nx > thr) { g = k; hit = true; break; }
    cum = nx;
  }
  if (!hit) cum -= (double)gs;                             // the last group
  const int c1 = min(nch, (g + 1) * KDE_MT_GROUP);
  int ch = c1 - 1;
  float cs = 0.f;
  hit = false;
  for (int c = g * KDE_MT_GROUP; c < c1; ++c) {          // the chunk inside it
    cs = poly(row[c]);
    const double nx = cum + (double)cs;
    if (nx > thr) { ch = c; hit = true; break; }
    cum = nx;
  }
  if (!hit) cum -= (double)cs;                             // the group's last chunk
  const int j0 = min(M, ch * per), j1 = min(M, j0 + per);
  const float4* __restrict__ rev = rec + (((M + 15) >> 4) * 16 + KDE_REC_TAIL);
  return kde_scan(rec, rev, M, j0, j1, (float)(thr - cum), cs,
                  [&](const float4 r) { return fmaf(r.y, -1.f, fmaf(r.x, xb0, -0.f)); });
}

// Latent non-root KDE node, parent dims 1..3: index ~ softmax_j log K_p (kde.py:172-178).
// Pass 1 (MFMA): per-chunk weight sums -> scr[chunk][lane]; pass 2 (VALU replica): locate the
// chunk holding u * total, scan it.  All-underflow particles (every weight 0) redo the sums on
// VALU relative to their largest weight.
// lsp (out): ln sum_j K_p(x, y_j) -- the node's own log-density denominator (kde.py:141-146), from
// pass 1's total, ln(tot) + (sigma - |x'|^2) ln 2 in every form (factored, full, rescued,
// precomputed, moment table); NaN when pass 1 gave no positive total
__device__ __forceinline__ int kde_index_mfma(const vbn_walk_args& A, const vbn_step& st, const Lane& L,
                                              float ucat, float c_p, float& lsp) {
  const int M = st.k, nf = st.aux0, lane = L.lane;
  const int cb = kde_cb(M);
  int slots[4] = {0, 0, 0, 0};
  float scl[4] = {c_p, c_p, c_p, c_p};
  for (int f = 0; f < nf; ++f) slots[f] = L.ic[st.in_off + f];
  double tot = 0.0;
  float xv[4] = {0.f, 0.f, 0.f, 0.f};
  const float negsq = kde_own(L, slots, scl, nf, xv);
  const bool pre = (st.flags & VBN_F_PRECOMP) != 0;
  // per-point records (4 weight-0 rows before the first point), then the reversed copy
  const float4* __restrict__ rec = reinterpret_cast<const float4*>(L.P + st.reserved[3]) + 4;
  if (nf == 1 && KDE_MT(st) >= 0 && !(st.flags & (VBN_F_PRECOMP | VBN_F_PRE_OUT)) &&
      __all(-negsq <= KDE_FFORM_MAX)) {               // a one-feature node with a moment table
    float mtot = 0.f;
    const int idx = kde_index_moments(L.P + KDE_MT(st), 2.f * xv[0], ucat, rec, M, mtot);
    if (idx >= 0) {                                   // the whole wave took it
      if (mtot > 0.f) lsp = __logf(mtot) + negsq * VBN_LN2_F;   // factored form (sigma 0)
      wave_sync();
      return idx;
    }
  }
  float shift = 0.f;                                  // sigma: the sums are of exp2(a' - sigma)
  // pass 1 also keeps each chunk's first-half sum (a private array, kde_sub_blocks), so the
  // scan covers the half holding the threshold: at most a quarter chunk instead of a half
  bool halves = false;
#ifndef VBN_ABL_NOHALVES
  float hs[KDE_CHUNKS * (KDE_NSUB - 1)];
#endif
  if (pre) {                                          // pass 1 of this sample / query, pre-pass
    if (st.flags & VBN_F_PRECOMP_Q) {
      const cfloat* q = precomp_qrow(A, st, L);
      for (int ch = 0; ch < KDE_CHUNKS; ++ch) {
        const float cs = q[ch];
        L.scr[ch * WAVE + lane] = cs;
        tot += (double)cs;
      }
      shift = q[KDE_CHUNKS];
    } else {
      const float* __restrict__ q = precomp_row(A, st, L);
      for (int ch = 0; ch < KDE_CHUNKS; ++ch) {
        const float cs = q[ch];
        L.scr[ch * WAVE + lane] = cs;
        tot += (double)cs;
      }
      shift = q[KDE_CHUNKS];
    }
  } else
#ifdef VBN_ABL_NOP1
  if (true) {
    for (int ch = 0; ch < KDE_CHUNKS; ++ch) { L.scr[ch * WAVE + lane] = 1.f; tot += 1.0; }
  } else
#endif
  {
    const bf16x8* __restrict__ pa = reinterpret_cast<const bf16x8*>(L.P + st.reserved[1]) + lane;
    const bool fform = __all(-negsq <= KDE_FFORM_MAX);
    shift = fform ? 0.f : -negsq;
#ifndef VBN_ABL_NOHALVES
    // chunks of >= KDE_HALF_MIN 32-point blocks only: shorter chunks scan little, and the
    // sums' 64 B of scratch per particle then cost fabric traffic for no time (cfg5, M = 4096:
    // 8 blocks per chunk, 58.9 ms either way, 27 vs 7 GB per launch)
    float* hsp = ((st.flags & VBN_F_PRE_OUT) || (cb >> 1) < KDE_HALF_MIN) ? nullptr : hs;
    halves = hsp != nullptr;
#else
    float* hsp = nullptr;
#endif
    if (nf == 1)
      tot = kde_pass1<1, 1>(pa, cb >> 1, L, slots, scl, nf, fform, hsp);
    else if (nf == 2 && fform)
      tot = kde_pass1<1, 2>(pa, cb >> 1, L, slots, scl, nf, fform, hsp);
    else
      tot = kde_pass1<2, 2>(pa, cb >> 1, L, slots, scl, nf, fform, hsp);
  }
  const int nfr = nf;                                 // replica form of the pass-1 elements
  const float xb0 = 2.f * xv[0], xb1 = 2.f * xv[1], xb2 = 2.f * xv[2];
  if (!pre && !(tot > 0.0)) {                         // every weight underflowed (or NaN parent)
    halves = false;
    float amax = -INFINITY;
    for (int j = 0; j < M; ++j) amax = fmaxf(amax, kde_arg_rec(rec[j], xb0, xb1, xb2, 0.f, nfr));
    shift = amax;
    tot = 0.0;
    for (int ch = 0; ch < KDE_CHUNKS; ++ch) {
      const int j0 = min(M, ch * cb * 16), j1 = min(M, j0 + cb * 16);
      float cs = 0.f;
      for (int j = j0; j < j1; ++j)
        cs += __builtin_amdgcn_exp2f(kde_arg_rec(rec[j], xb0, xb1, xb2, 0.f, nfr) - shift);
      L.scr[ch * WAVE + lane] = cs;
      tot += (double)cs;
    }
  }
  if (tot > 0.0) lsp = __logf((float)tot) + (shift + negsq) * VBN_LN2_F;
  if (st.flags & VBN_F_PRE_OUT) {                    // pre-pass: pass 1's result is the output
    for (int c = 0; c < KDE_CHUNKS; ++c) vwrite(L, st.out_col + c, L.scr[c * WAVE + lane]);
    vwrite(L, st.out_col + KDE_CHUNKS, shift);
    wave_sync();
    return -1;
  }
  const double thr = (double)ucat * tot;
  double cum = 0.0;
  int ch = KDE_CHUNKS - 1;
  for (int c2 = 0; c2 < KDE_CHUNKS; ++c2) {
    const double nx = cum + (double)L.scr[c2 * WAVE + lane];
    if (nx > thr) { ch = c2; break; }
    cum = nx;
  }
  const int j0 = min(M, ch * cb * 16), j1 = min(M, j0 + cb * 16);
#ifdef VBN_ABL_NOSCAN
  wave_sync();
  return min(j0, M - 1);
#endif
  float rem = (float)(thr - cum);
  float csum = L.scr[ch * WAVE + lane];
  int jlo = j0, jhi = j1;
#ifndef VBN_ABL_NOHALVES
  if (halves) {                                       // the sub-chunk holding thr
    const double rd = thr - cum;
    float plo = 0.f, phi = csum;
    int klo = 0, khi = KDE_NSUB;
#pragma unroll
    for (int k = 1; k < KDE_NSUB; ++k) {
      const float pk = hs[ch * (KDE_NSUB - 1) + k - 1];
      if (rd >= (double)pk) { klo = k; plo = pk; }
      else if (khi == KDE_NSUB) { khi = k; phi = pk; }
    }
    const int cb32 = cb >> 1;
    jlo = klo ? min(M, j0 + 32 * kde_sub_blocks(cb32, klo)) : j0;
    jhi = khi < KDE_NSUB ? min(M, j0 + 32 * kde_sub_blocks(cb32, khi)) : j1;
    rem = (float)(rd - (double)plo);
    csum = phi - plo;
  }
#endif
  const float4* __restrict__ rev = rec + (((M + 15) >> 4) * 16 + KDE_REC_TAIL);
  int idx;
  // the replica chain a' = 2 x'.y' - |y'|^2 per feature count, compile-time (kde_arg_rec with
  // no -|x'|^2 term: sigma carries it in the full form)
  // (the shift enters the chain as its addend: -0 in the factored form, so the same values)
  const float nsh = -shift;
  if (nfr == 1)
    idx = kde_scan(rec, rev, M, jlo, jhi, rem, csum,
                   [&](const float4 r) { return fmaf(r.y, -1.f, fmaf(r.x, xb0, nsh)); });
  else if (nfr == 2)
    idx = kde_scan(rec, rev, M, jlo, jhi, rem, csum, [&](const float4 r) {
      return fmaf(r.z, -1.f, fmaf(r.y, xb1, fmaf(r.x, xb0, nsh)));
    });
  else
    idx = kde_scan(rec, rev, M, jlo, jhi, rem, csum, [&](const float4 r) {
      return fmaf(r.w, -1.f, fmaf(r.z, xb2, fmaf(r.y, xb1, fmaf(r.x, xb0, nsh))));
    });
  wave_sync();
  return idx;
}

// log p(x | parents) of a KDE node on MFMA (kde.py:114-146):
//   root:     LSE_j log K_y - log M
//   non-root: LSE_j (log K_p + log K_y) - LSE_j log K_p
// pack kq (parent features) and kqy (parent ++ target features, scales c_p / c_y).  Returns
// false (nothing added) when a sum underflows; the caller then takes the shifted VALU path.
__device__ __forceinline__ bool kde_logp_mfma(const vbn_step& st, const Lane& L, bool root, float c_p,
                                              float c_y, float cy, float log_n, float& lp, float lsp) {
  const int M = st.k, dp = st.aux0, D = st.out_dim, lane = L.lane;
  // the blocks holding points (a whole number of KDE_PF blocks), not the chunk-padded pack: the
  // blocks past them hold only weight-0 padding, whose +0 terms leave every sum unchanged
  const int nb32 = min((KDE_CHUNKS * kde_cb(M)) >> 1, (((M + 31) >> 5) + KDE_PF - 1) / KDE_PF * KDE_PF);
  int slots[4] = {0, 0, 0, 0};
  float scl[4] = {c_p, c_p, c_p, c_p};
  for (int f = 0; f < dp; ++f) slots[f] = L.ic[st.in_off + f];
  for (int d = 0; d < D; ++d) { slots[dp + d] = st.out_col + d; scl[dp + d] = c_y; }
  const int ny = dp + D;
  // factored sums (kde_pass1) when no lane's |x'|^2 can overflow them: ln of a full-form sum =
  // ln(factored sum) - |x'|^2 ln 2
  float xv[4];
  const float sq_y = -kde_own(L, slots, scl, ny, xv);
  const float sq_p = root ? 0.f : -kde_own(L, slots, scl, dp, xv);
  const bool fform = __all(sq_y <= KDE_FFORM_MAX);
  const bf16x8* __restrict__ pay = reinterpret_cast<const bf16x8*>(L.P + st.reserved[2]) + lane;
  const float sy = kde_sums_nf(pay, nb32, L, slots, scl, ny, fform);
  constexpr float LN2 = 0.69314718055994531f;
#ifndef VBN_ABL_NOLSP
  // a sampled node's denominator is its own pass 1's total (kde_index_mfma lsp): every lane of
  // the wave has it, so the parent-feature pass is not run again (cfg4's target: M exps per
  // particle)
  if (!root && __all(lsp == lsp)) {
    wave_sync();
    if (!(sy > 0.f)) return false;
    lp += ((__logf(sy) - (fform ? sq_y * LN2 : 0.f)) - lsp) + cy;
    return true;
  }
#endif
  float sp = 1.f;
  if (!root) {
    const bf16x8* __restrict__ pa = reinterpret_cast<const bf16x8*>(L.P + st.reserved[1]) + lane;
    sp = kde_sums_nf(pa, nb32, L, slots, scl, dp, fform);
  }
  wave_sync();
  if (!(sy > 0.f) || !(sp > 0.f)) return false;
  const float corr = fform ? (root ? sq_y : sq_y - sq_p) * LN2 : 0.f;
  lp += root ? ((__logf(sy) - corr) + cy - log_n) : (((__logf(sy) - __logf(sp)) - corr) + cy);
  return true;
}

// ---- pairwise kernel weights on VALU (alternative path, VBN_F_KDE_VALU) ---------------------
// -|x' - y'|^2 with packed f32 VALU (v_pk_add / v_pk_mul / v_pk_fma on two points per lane),
// points wave-uniform from scalar loads.  Measured on MI355X (cfg4, 64-node KDE, M = 10k,
// 4096 x 1024 particles): 253 ms per walk vs 245 ms with the MFMA distance tile (and 266 ms
// with the scalar loads software-pipelined), so the MFMA tile is the default.
// Pack kv (plan.py _kde_pack_valu): [KDE_CHUNKS * csz / 8][NF][8] fp32, padding points
// y' = 1e15 (weight 0).  Chunk ch = points [ch * csz, (ch + 1) * csz).
__device__ __forceinline__ int kde_csz(int M) { return (((M + KDE_CHUNKS - 1) / KDE_CHUNKS) + 7) & ~7; }

// -|x' - y'|^2 of one point record r = (y'_0, y'_1, y'_2, .); same operations, same order as
// the packed pass (bit-identical per element)
template <int NF>
__device__ __forceinline__ float kde_arg_valu(const float (&xv)[4], const float4 r) {
#pragma clang fp contract(off)
  const float d0 = xv[0] - r.x;
  float a = d0 * d0;
  if (NF > 1) { const float d1 = xv[1] - r.y; a = fmaf(d1, d1, a); }
  if (NF > 2) { const float d2 = xv[2] - r.z; a = fmaf(d2, d2, a); }
  return -a;
}

template <int NF>
__device__ __forceinline__ int kde_index_valu(const vbn_walk_args& A, const vbn_step& st, const Lane& L,
                                              float ucat, float c_p) {
#pragma clang fp contract(off)
  const float* __restrict__ kv = L.P + st.reserved[4];
  const int M = st.k, lane = L.lane, csz = kde_csz(M);
  float xv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int f = 0; f < NF; ++f) xv[f] = c_p * vread(L, L.ic[st.in_off + f]);
  f32x2 xp[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) xp[f] = f32x2{xv[f], xv[f]};
  double tot = 0.0;
  for (int ch = 0; ch < KDE_CHUNKS; ++ch) {
    const float* __restrict__ blk = kv + (int64_t)(ch * (csz >> 3)) * (NF * 8);
    f32x2 acc = f32x2{0.f, 0.f};
    for (int b = 0; b < (csz >> 3); ++b, blk += NF * 8) {
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        const f32x2 d0 = xp[0] - f32x2{blk[i], blk[i + 1]};
        f32x2 a = d0 * d0;
        if (NF > 1) {
          const f32x2 d1 = xp[1] - f32x2{blk[8 + i], blk[8 + i + 1]};
          a = __builtin_elementwise_fma(d1, d1, a);
        }
        if (NF > 2) {
          const f32x2 d2 = xp[2] - f32x2{blk[16 + i], blk[16 + i + 1]};
          a = __builtin_elementwise_fma(d2, d2, a);
        }
        acc += f32x2{__builtin_amdgcn_exp2f(-a.x), __builtin_amdgcn_exp2f(-a.y)};
      }
    }
    const float cs = acc.x + acc.y;
    L.scr[ch * WAVE + lane] = cs;
    tot += (double)cs;
  }
  // per-point records (4 weight-0 rows before the first point), then the reversed copy
  const float4* __restrict__ rec = reinterpret_cast<const float4*>(L.P + st.reserved[3]) + 4;
  float shift = 0.f;
  if (!(tot > 0.0)) {                                 // every weight underflowed (or NaN parent)
    float amax = -INFINITY;
    for (int j = 0; j < M; ++j) amax = fmaxf(amax, kde_arg_valu<NF>(xv, rec[j]));
    shift = amax;
    tot = 0.0;
    for (int ch = 0; ch < KDE_CHUNKS; ++ch) {
      const int j0 = min(M, ch * csz), j1 = min(M, j0 + csz);
      float cs = 0.f;
      for (int j = j0; j < j1; ++j) cs += __builtin_amdgcn_exp2f(kde_arg_valu<NF>(xv, rec[j]) - shift);
      L.scr[ch * WAVE + lane] = cs;
      tot += (double)cs;
    }
  }
  const double thr = (double)ucat * tot;
  double cum = 0.0;
  int ch = KDE_CHUNKS - 1;
  for (int c2 = 0; c2 < KDE_CHUNKS; ++c2) {
    const double nx = cum + (double)L.scr[c2 * WAVE + lane];
    if (nx > thr) { ch = c2; break; }
    cum = nx;
  }
  const int j0 = min(M, ch * csz), j1 = min(M, j0 + csz);
  const float rem = (float)(thr - cum);
  const float csum = L.scr[ch * WAVE + lane];
  const float4* __restrict__ rev = rec + (((M + 15) >> 4) * 16 + KDE_REC_TAIL);
  const int idx = kde_scan(rec, rev, M, j0, j1, rem, csum,
                           [&](const float4 r) { return kde_arg_valu<NF>(xv, r) - shift; });
  wave_sync();
  return idx;
}

template <int DP, int DY>
__device__ __forceinline__ void step_kde_t(const vbn_walk_args& A, const vbn_step& st, const Lane& L, float& lp) {
#pragma clang fp contract(off)
  const float* __restrict__ P = L.P;
  const float* __restrict__ pts = P + st.off_pts;
  const int M = st.k, dp = DP >= 0 ? DP : st.aux0, stride = st.aux1, D = DY > 0 ? DY : st.out_dim;
  const cfloat* t = CP(P + st.off_tail);
  const float inv_sp = t[0], inv_sy = t[1], noise_scale = t[2], cy = t[3], log_n = t[4];
  const float c_p = t[5], c_y = t[6];
  const bool root = (st.flags & VBN_F_ROOT) != 0;
  const int lane = L.lane;
  float pv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < (DP > 0 ? DP : 0); ++i) pv[i] = vread(L, L.ic[st.in_off + i]);

  float lsp = __int_as_float(0x7fc00000);            // the sampling pass's ln sum_j K_p (NaN: none)
  if (st.role == VBN_ROLE_LATENT) {
    const float ucat = draw_uniforms(A, st, 0, L).x;
    int idx;
    if (root) {
      idx = min((int)(ucat * (float)M), M - 1);             // randint(0, M)
    } else if (st.reserved[4] >= 0 && (st.flags & VBN_F_KDE_VALU)) {
      idx = st.aux0 == 1 ? kde_index_valu<1>(A, st, L, ucat, c_p)
          : (st.aux0 == 2 ? kde_index_valu<2>(A, st, L, ucat, c_p) : kde_index_valu<3>(A, st, L, ucat, c_p));
    } else if (st.reserved[1] >= 0) {
      idx = kde_index_mfma(A, st, L, ucat, c_p, lsp);
      if (st.flags & VBN_F_PRE_OUT) return;            // pre-pass: sums written, no sample
    } else {
      // pass 1: per-chunk weight sums -> scr[chunk][lane]
      const int csz = (M + KDE_CHUNKS - 1) / KDE_CHUNKS;
      double tot = 0.0;
      float qmin = INFINITY;
      for (int ch = 0; ch < KDE_CHUNKS; ++ch) {
        const int j0 = ch * csz, j1 = min(M, j0 + csz);
        float cs = 0.f;
        for (int j = j0; j < j1; ++j) {
          const float q = kde_qp<DP>(pts + (int64_t)j * stride, pv, inv_sp, dp, A, st, L);
          qmin = fminf(qmin, q);
          cs += __expf(-0.5f * q);
        }
        L.scr[ch * WAVE + lane] = cs;
        tot += (double)cs;
      }
      float shift = 0.f;
      if (!(tot > 0.0)) {                                 // all weights underflowed
        shift = qmin;
        tot = 0.0;
        for (int ch = 0; ch < KDE_CHUNKS; ++ch) {
          const int j0 = ch * csz, j1 = min(M, j0 + csz);
          float cs = 0.f;
          for (int j = j0; j < j1; ++j)
            cs += __expf(-0.5f * (kde_qp<DP>(pts + (int64_t)j * stride, pv, inv_sp, dp, A, st, L) - shift));
          L.scr[ch * WAVE + lane] = cs;
          tot += (double)cs;
        }
      }
      // pass 2: locate the chunk, then scan inside it (per-lane chunk; vector loads)
      const double thr = (double)ucat * tot;
      double cum = 0.0;
      int ch = KDE_CHUNKS - 1;
      for (int c2 = 0; c2 < KDE_CHUNKS; ++c2) {
        const double nx = cum + (double)L.scr[c2 * WAVE + lane];
        if (nx > thr) { ch = c2; break; }
        cum = nx;
      }
      const int j0 = ch * csz, j1 = min(M, j0 + csz);
      const float rem = (float)(thr - cum);
      float cs = 0.f;
      idx = max(j1 - 1, 0);
      for (int j = j0; j < j1; ++j) {
        cs += __expf(-0.5f * (kde_qp<DP>(pts + (int64_t)j * stride, pv, inv_sp, dp, A, st, L) - shift));
        if (cs > rem) { idx = j; break; }
      }
      wave_sync();
    }
    for (int d = 0; d < D; ++d) {
      const float sel = pts[(int64_t)idx * stride + dp + d];
      vwrite(L, st.out_col + d, sel + draw_normal(A, st, d, L) * noise_scale);
    }
  } else {
    for (int d = 0; d < D; ++d) vwrite(L, st.out_col + d, node_fixed(A, st, d, L));
  }

  if ((st.flags & VBN_F_LOGP) && st.reserved[2] >= 0 && (root || st.reserved[1] >= 0)) {
    wave_sync();
    if (kde_logp_mfma(st, L, root, c_p, c_y, cy, log_n, lp, lsp)) return;
  }
  if (st.flags & VBN_F_LOGP) {
    const float x0 = NODE_X(0);
    float sy = 0.f, sp = 0.f, qymin = INFINITY, qpmin = INFINITY, qsmin = INFINITY;
    for (int j = 0; j < M; ++j) {
      const float* pt = pts + (int64_t)j * stride;
      const float qy = kde_qy<DY>(pt + dp, x0, inv_sy, D, st, L);
      if (root) {
        sy += __expf(-0.5f * qy);
        qymin = fminf(qymin, qy);
      } else {
        const float qp = kde_qp<DP>(pt, pv, inv_sp, dp, A, st, L);
        sp += __expf(-0.5f * qp);
        sy += __expf(-0.5f * (qp + qy));
        qpmin = fminf(qpmin, qp);
        qsmin = fminf(qsmin, qp + qy);
      }
    }
    float sh_y = 0.f, sh_p = 0.f;
    if (!(sy > 0.f) || (!root && !(sp > 0.f))) {   // underflow: re-sum relative to the minimum
      sh_y = root ? qymin : qsmin;
      sh_p = qpmin;
      sy = 0.f;
      sp = 0.f;
      for (int j = 0; j < M; ++j) {
        const float* pt = pts + (int64_t)j * stride;
        const float qy = kde_qy<DY>(pt + dp, x0, inv_sy, D, st, L);
        if (root) {
          sy += __expf(-0.5f * (qy - sh_y));
        } else {
          const float qp = kde_qp<DP>(pt, pv, inv_sp, dp, A, st, L);
          sp += __expf(-0.5f * (qp - sh_p));
          sy += __expf(-0.5f * (qp + qy - sh_y));
        }
      }
    }
    const float ls_y = logf(sy) - 0.5f * sh_y;
    if (root) {
      lp += ls_y + cy - log_n;
    } else {
      const float ls_p = logf(sp) - 0.5f * sh_p;
      lp += (ls_y - ls_p) + cy;
    }
  }
}

__device__ __forceinline__ void step_kde(const vbn_walk_args& A, const vbn_step& st, const Lane& L, float& lp) {
  if (st.out_dim == 1) {
    switch (st.aux0) {
      case 0: step_kde_t<0, 1>(A, st, L, lp); return;
      case 1: step_kde_t<1, 1>(A, st, L, lp); return;
      case 2: step_kde_t<2, 1>(A, st, L, lp); return;
      case 3: step_kde_t<3, 1>(A, st, L, lp); return;
      default: break;
    }
  }
  step_kde_t<-1, -1>(A, st, L, lp);
}

// ------------------------------------------------------------------------------------------
// Gibbs sweep steps (gibbs.py:40-87): lanes 8c .. 8c+7 hold chain c's 8 candidates
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void gibbs_select(const vbn_walk_args& A, const vbn_step& st, Lane& L, float lp) {
  const int lane = L.lane, g0 = lane & ~7;
  float m = fmaxf(lp, __shfl_xor(lp, 1));
  m = fmaxf(m, __shfl_xor(m, 2));
  m = fmaxf(m, __shfl_xor(m, 4));
  const float e = __expf(lp - m);                       // softmax(log_score, 1) (79)
  float se = e + __shfl_xor(e, 1);
  se += __shfl_xor(se, 2);
  se += __shfl_xor(se, 4);
  float pk[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) pk[k] = __shfl(e, g0 + k) / se;
  // one uniform per chain (candidate lane 0's draw), multinomial(weights, 1) (80); without
  // injected noise it comes from the node's own SELECT stream, which no candidate draw uses
  const int s_keep = L.s;
  L.s = 0;
  const float u = (!L.noiseless && A.noise) ? draw_uniforms(A, st, 0, L).x : u01(rng_words(A, st, 0, RNG_SELECT, L).x);
  L.s = s_keep;
  const int idx = inv_cdf(8, u, [&](int k) { return pk[k]; });
  for (int d = 0; d < st.out_dim; ++d) {
    const float v = __shfl(vread(L, st.out_col + d), g0 + idx);
    wave_sync();
    vwrite(L, st.out_col + d, v);                        // chosen candidate (81-82)
  }
}

__device__ __forceinline__ void gibbs_collect(const vbn_walk_args& A, const vbn_step& st, const Lane& L) {
  const int it = L.iter, burn = A.gibbs_burn_in, thin = max(A.gibbs_thin, 1);
  if (it < burn || (it - burn) % thin != 0 || L.s != 0 || !L.valid || (L.mirror && L.lane >= 32)) return;  // 83-87
  const int n_collect = (A.gibbs_iters - burn + thin - 1) / thin;
  const int k = (it - burn) / thin;
  for (int d = 0; d < st.out_dim; ++d)
    A.out_x[(L.b * n_collect + k) * A.n_out_cols + d] = vread(L, st.out_col + d);
}

// ------------------------------------------------------------------------------------------
// the walk
// ------------------------------------------------------------------------------------------
// One step of the walk for the wave's 64 particles.
// KM: bit0 gaussian_nn, bit1 linear_gaussian, bit2 mdn, bit3 kde, bit4 softmax_nn,
// bit5 non-relu activations.  Each instantiation only carries the code (and registers) of
// the CPD kinds a plan uses.
template <unsigned KM>
__device__ __forceinline__ void walk_step(const vbn_walk_args& A, const vbn_step& st, Lane& L, float& lp) {
  if (st.role == VBN_ROLE_SKIP) return;
  if (!L.lean && (st.flags & VBN_F_LPRESET)) lp = 0.f;
  if (!L.lean && st.role == VBN_ROLE_SELECT) {        // Gibbs roles: not in lean walks
    gibbs_select(A, st, L, lp);
    wave_sync();
    return;
  }
  if (!L.lean && st.role == VBN_ROLE_COLLECT) {
    gibbs_collect(A, st, L);
    return;
  }
  if ((st.flags & VBN_F_PRE_OUT) && st.kind != VBN_KIND_KDE) {   // shared-sample pre-pass: the
    if constexpr ((KM & 21u) != 0) {                                 // NN CPD's head outputs
      if (st.kind == VBN_KIND_GAUSSIAN_NN && st.out_dim == 1) run_mlp<KM, 2>(A, st, L, [] {});
      else run_mlp<KM>(A, st, L, [] {});
      for (int j = 0; j < st.n_out; ++j) vwrite(L, st.out_col + j, L.scr[j * WAVE + L.lane]);
    }
    wave_sync();
    return;
  }
  if (st.role == VBN_ROLE_FIXED && !(st.flags & VBN_F_LOGP)) {   // evidence / do: value only
    for (int d = 0; d < st.out_dim; ++d) vwrite(L, st.out_col + d, node_fixed(A, st, d, L));
    wave_sync();
    return;
  }
  switch (st.kind) {
    case VBN_KIND_GAUSSIAN_NN: if constexpr ((KM & 1) != 0) step_gaussian_nn<KM>(A, st, L, lp); break;
    case VBN_KIND_LINEAR_GAUSSIAN: if constexpr ((KM & 2) != 0) step_linear_gaussian(A, st, L, lp); break;
    case VBN_KIND_MDN: if constexpr ((KM & 4) != 0) step_mdn<KM>(A, st, L, lp); break;
    case VBN_KIND_KDE: if constexpr ((KM & 8) != 0) step_kde(A, st, L, lp); break;
    default: if constexpr ((KM & 16) != 0) step_softmax_nn<KM>(A, st, L, lp); break;
  }
  wave_sync();
}

typedef __attribute__((address_space(3))) void lds_void;
// Staged walks (kind sets of gaussian_nn / linear_gaussian only): NN weight blocks are DMA'd
// into LDS one step ahead and shared by the 4 waves of a workgroup, one barrier per step.
// Measured on MI355X (walk ms, staged vs direct): cfg2 1.22 vs 1.35; with mdn/softmax_nn heads
// (cfg3) 4.43 vs 4.26 and with KDE nodes (cfg5) 186 vs 166 (per-wave work varies by node, the
// barrier waits for the slowest wave) -- those kind sets read the blob straight (L1/L2).
#ifndef VBN_STAGE
#define VBN_STAGE 1
#endif
__host__ __device__ constexpr bool staged_kinds(unsigned km) { return VBN_STAGE && (km & 28u) == 0; }
#define WG_MAX_WAVES 4
#define WBLK_CHUNK 256   // floats per global_load_lds_dwordx4 wave instruction (64 lanes x 16 B)

// Stage step j's NN weight block into LDS weight buffer ``buf``: the workgroup's waves split
// its 1-KiB chunks, one global_load_lds_dwordx4 each (no VGPRs; completion is waited for by
// step_barrier before the step that reads it).
__device__ __forceinline__ void stage_block(const vbn_walk_args& A, const vbn_step* __restrict__ steps,
                                            const float* __restrict__ params, float* wbuf, int j, int buf,
                                            int wave, int nw, int lane) {
  const int off = steps[j].reserved[5], len = steps[j].reserved[6];
  if (len <= 0) return;
  float* dst = wbuf + buf * A.wbuf_floats;
  for (int c = wave; c * WBLK_CHUNK < len; c += nw)
    __builtin_amdgcn_global_load_lds((const void*)(params + off + c * WBLK_CHUNK + lane * 4),
                                     (lds_void*)(dst + c * WBLK_CHUNK), 16, 0, 0);
}

// first step >= j that runs an MLP (has a weight block), or -1
__device__ __forceinline__ int first_mlp(const vbn_step* __restrict__ steps, int j, int n) {
  for (; j < n; ++j)
    if (CI(steps)[j * (int)(sizeof(vbn_step) / 4) + (int)(__builtin_offsetof(vbn_step, reserved) / 4) + 6] > 0) return j;
  return -1;
}

// start of an MLP step: this wave's LDS-DMA of the step's block has landed, every wave of the
// workgroup is done with the buffer the next MLP step's prefetch overwrites
__device__ __forceinline__ void step_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef VBN_ABL_NOBAR
  return;
#endif
  __syncthreads();
}

// (ABI v13) Posterior-summary partials of VBN._posterior_stats (vbn.py:495-503) fused into an
// MCM walk's epilogue: the wave's 64 particles all belong to query L.b (n_samples % 64 == 0), so
// it reduces their weights w = pdf (nan / inf -> 0, clamped >= 0) and target values in float64
// with xor butterflies (every lane ends with the same sums) and lane 0 writes one row of
// vbn_walk_args.stats_part: [W, Q, per output column: m_w, M2_w, m_u, M2_u] (two-pass inside the
// wave: the mean first, then the centred second moment around it).  A zero-weight wave keeps
// m_w = sum w x (0, or NaN when a sample is NaN as in the reference's 0 * NaN).
// vbn_hip_posterior_stats_merge combines a query's S / 64 rows.
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ void stats_partials(const vbn_walk_args& A, const Lane& L, float pdf) {
  const int D = A.n_out_cols;
  const double w = (pdf != pdf || pdf == INFINITY || pdf == -INFINITY) ? 0.0 : (double)fmaxf(pdf, 0.f);
  const double W = wave_sum_f64(w), Q = wave_sum_f64(w * w);
  const int stride = 2 + 4 * D;
  double* row = A.stats_part + ((int64_t)L.b * (A.n_samples >> 6) + (L.s >> 6)) * stride;
  if (L.lane == 0) {
    row[0] = W;
    row[1] = Q;
  }
  for (int d = 0; d < D; ++d) {
    const double x = (double)vread(L, A.out_cols[d]);
    const double sx = wave_sum_f64(w * x);
    const double mw = W > 0.0 ? sx / W : sx;
    const double cw = x - mw;
    const double m2w = wave_sum_f64(w * (cw * cw));
    const double mu = wave_sum_f64(x) * (1.0 / 64.0);
    const double cu = x - mu;
    const double m2u = wave_sum_f64(cu * cu);
    if (L.lane == 0) {
      row[2 + 4 * d] = mw;
      row[3 + 4 * d] = m2w;
      row[4 + 4 * d] = mu;
      row[5 + 4 * d] = m2u;
    }
  }
}

// The walk.  A workgroup = nw (1, 2 or 4; blockDim.x / 64) waves, each owning 64 consecutive
// particles with its own LDS value slots; the waves walk the same step table in lockstep (one
// barrier per step) and share two LDS weight buffers: while step i runs on buffer i & 1, step
// i + 1's MLP weights are DMA'd into the other one (one memory latency per step, hidden
// behind the step's compute, and one copy per workgroup instead of per wave).
#ifndef VBN_WPE
#define VBN_WPE 4
#endif
template <unsigned KM>
__global__ void __launch_bounds__(WG_MAX_WAVES * WAVE) __attribute__((amdgpu_waves_per_eu(VBN_WPE)))
vbn_walk_kernel(const vbn_walk_args A, const float* __restrict__ params, const vbn_step* __restrict__ steps,
                const int32_t* __restrict__ in_cols) {
  if (A.run_if && *A.run_if == 0) return;            // predicated launch, not needed (uniform)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nw = blockDim.x >> 6, wave = threadIdx.x >> 6;
  const int per_wave = (A.n_slots + (A.max_out > 0 ? A.max_out : 1)) * WAVE;
  float* wbuf = smem + nw * per_wave;
  Lane L;
  L.P = params;
  L.ic = in_cols;
  L.lane = threadIdx.x & (WAVE - 1);
  L.vals = smem + wave * per_wave;
  L.scr = L.vals + A.n_slots * WAVE;
  L.wb = wbuf;
  const int64_t total = A.n_queries * (int64_t)A.n_samples;
  // half-wave launches (wave_particles 32): lane l and l + 32 carry the same particle, so
  // every draw and value agrees; only the lower half writes, the MLPs run group 0 only
  L.mirror = (KM & 64) != 0;                         // host: wave_particles == 32
  L.lean = (KM & 128) != 0;                          // host: no noise, no state, not Gibbs
  L.noiseless = (KM & (128 | 256)) != 0;             // host: no injected draws
  L.bm_spare = 0.f;
  const int wp = L.mirror ? 32 : WAVE;
  L.wq = A.mode != VBN_MODE_GIBBS && (A.n_samples & (wp - 1)) == 0;
  const int64_t p_raw = ((int64_t)blockIdx.x * nw + wave) * wp + (L.lane & (wp - 1));
  const bool valid = p_raw < total;
  L.p = valid ? p_raw : total - 1;
  L.b = L.p / A.n_samples;
  L.s = (int)(L.p - L.b * A.n_samples);
  L.iter = 0;
  L.valid = valid;

  float lp = 0.f;
  if (!L.lean && A.state && (A.state_flags & 1)) {  // resume a segmented walk
    for (int c = 0; c < A.n_slots; ++c) vwrite(L, c, A.state[(int64_t)c * total + L.p]);
    lp = A.state[(int64_t)A.n_slots * total + L.p];
    wave_sync();
  }
  const int iters = (!L.lean && A.mode == VBN_MODE_GIBBS) ? A.gibbs_iters : 1;
  if constexpr (staged_kinds(KM)) {
  // Only MLP steps (wblk_len > 0) touch the weight buffers, so only they synchronise: MLP step
  // k waits for its block (DMA'd during MLP step k - 1), then, once every wave is past that
  // barrier (so done with the other buffer), DMAs MLP step k + 1's block into it.  The DMA
  // overlaps MLP step k and every root / evidence step up to k + 1.
  int par = 0;
  int nxt = first_mlp(steps, 0, A.n_steps);
  if (nxt >= 0) stage_block(A, steps, params, wbuf, nxt, 0, wave, nw, L.lane);
  for (int it = 0; it < iters; ++it) {
    L.iter = it;
    for (int i = 0; i < A.n_steps; ++i) {
      if (i == nxt) {
        step_barrier();
        nxt = first_mlp(steps, i + 1, A.n_steps);
        if (nxt < 0 && it + 1 < iters) nxt = first_mlp(steps, 0, A.n_steps);   // next sweep
        if (nxt >= 0) stage_block(A, steps, params, wbuf, nxt, par ^ 1, wave, nw, L.lane);
        L.wb = wbuf + par * A.wbuf_floats;
        par ^= 1;
      }
      walk_step<KM>(A, steps[i], L, lp);
    }
  }
  } else {
  (void)wbuf;
  for (int it = 0; it < iters; ++it) {
    L.iter = it;
    for (int i = 0; i < A.n_steps; ++i) {
      const vbn_step st = steps[i];
      L.wb = params + st.reserved[5];
      walk_step<KM>(A, st, L, lp);
    }
  }
  }
  if (!valid || (L.mirror && L.lane >= 32)) return;
  if (A.mode == VBN_MODE_GIBBS) return;                  // outputs written by COLLECT steps
  if (!L.lean && A.state && (A.state_flags & 2)) {
    for (int c = 0; c < A.n_slots; ++c) A.state[(int64_t)c * total + L.p] = vread(L, c);
    A.state[(int64_t)A.n_slots * total + L.p] = lp;
  }
  if (A.out_lp && A.mode != VBN_MODE_SAMPLE) A.out_lp[L.p] = (A.mode == VBN_MODE_MCM) ? __expf(lp) : lp;
  if (A.out_x) {
    for (int k = 0; k < A.n_out_cols; ++k)
      A.out_x[L.p * A.n_out_cols + k] = vread(L, A.out_cols[k]);
  }
  if (A.stats_part && A.mode == VBN_MODE_MCM && L.wq && !L.mirror) stats_partials(A, L, __expf(lp));
}

// Instantiated kind sets: bits 0-4 the CPD kinds walked, bit 5 non-relu activations, bit 6 the
// half-wave (mirror) launch (include/vbn_hip.h wave_particles = 32), bit 7 the lean walk (no
// injected draws, no segment state, not Gibbs: the production MCM / IS / LW / ancestral path;
// measured cfg2 1.215 -> 1.19 ms, SGPR spills 35 -> 0), bit 8 no injected draws (with bit 6: the
// production half-wave Gibbs sweeps; SGPR spills 34 -> 9), bit 9 the generic-MLP path (plans
// with hidden_dims other than (32, 32): only with the all-kinds set 63, so the out-of-line
// mlp_generic call never touches the hot instantiations' registers).  Each is compiled in its
// own object from walk_inst.hip (Makefile KIND_SETS must list the same values).
#define VBN_WALK_KIND_SETS(X) \
  X(1) X(2) X(3) X(4) X(8) X(16) X(20) X(23) X(31) X(63) \
  X(65) X(66) X(67) X(68) X(72) X(80) X(84) X(87) X(95) X(127) \
  X(129) X(130) X(131) X(132) X(136) X(144) X(148) X(151) X(159) X(191) \
  X(321) X(322) X(323) X(324) X(328) X(336) X(340) X(343) X(351) X(383) \
  X(575) X(639) X(703) X(895)
#define VBN_LAUNCHER_(K) vbn_launch_walk_km##K
#define VBN_LAUNCHER(K) VBN_LAUNCHER_(K)
