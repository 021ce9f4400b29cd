#pragma once
// vbn_walk_plan.h — the particle walk specialised for ONE step table (gfx950).
//
// The interpreter kernel (vbn_walk_kernel) reads each step's 32 fields, its parent-slot list
// and the LDS weight-buffer schedule from memory at run time and dispatches on role / kind /
// flags per step.  Here the step table is a compile-time constant: every field folds to an
// immediate, role / kind / flag branches disappear, the staging schedule (which block goes
// into which LDS buffer before which step) is computed by the compiler, and the steps are
// straight-line code the scheduler can overlap across node boundaries.  Same device
// functions, same operations in the same order: bit-identical outputs to the interpreter.
//
// The including translation unit defines, before including this header:
//   VBN_PLAN_N_STEPS                          number of steps
//   constexpr vbn_step VBN_PLAN_STEPS[]       the step table (vectorizedbayesiannetwork_amd/plan.py)
//   __constant__ int32_t VBN_PLAN_IC[]        the parent-slot list (in_cols)
// and instantiates vbn_walk_plan_body<KM> in its own __global__ kernel.  The package compiles
// such a unit at run time with hiprtc per (plan, kind set) (vectorizedbayesiannetwork_amd/jit.py)
// and launches it through vbn_hip_walk_module (include/vbn_hip.h), for every walk form the
// interpreter has (lean, half-wave, Gibbs sweeps, injected draws, segment state).
#include "vbn_walk_impl.h"

template <typename T, T... I>
struct vbn_seq {};

constexpr int vbn_plan_next_mlp(int j) {
  for (; j < VBN_PLAN_N_STEPS; ++j)
    if (VBN_PLAN_STEPS[j].reserved[6] > 0) return j;
  return -1;
}

// LDS weight buffer step i's block lives in when the table runs once: MLP steps alternate 0, 1, 0, ...
constexpr int vbn_plan_parity(int i) {
  int par = 0;
  for (int j = 0; j < i; ++j)
    if (VBN_PLAN_STEPS[j].reserved[6] > 0) par ^= 1;
  return par;
}

template <int J>
__device__ __forceinline__ void vbn_plan_stage(const vbn_walk_args& A, const float* __restrict__ params, float* wbuf,
                                               int buf, int wave, int nw, int lane) {
  constexpr int off = VBN_PLAN_STEPS[J].reserved[5], len = VBN_PLAN_STEPS[J].reserved[6];
  float* dst = wbuf + buf * A.wbuf_floats;
  for (int c = wave; c * WBLK_CHUNK < len; c += nw)
    __builtin_amdgcn_global_load_lds((const void*)(params + off + c * WBLK_CHUNK + lane * 4),
                                     (lds_void*)(dst + c * WBLK_CHUNK), 16, 0, 0);
}

// One step.  Staged kind sets: an MLP step waits for its block (DMA'd one MLP step earlier),
// stages the next MLP step's block into the other buffer -- across the sweep boundary when
// another Gibbs sweep follows (``more``) -- and runs on its buffer ``par``; the same schedule
// as vbn_walk_kernel's, with every index known at compile time.
template <unsigned KM, int I>
__device__ __forceinline__ void vbn_plan_step(const vbn_walk_args& A, const float* __restrict__ params, float* wbuf,
                                              int wave, int nw, Lane& L, float& lp, int& par, bool more) {
  constexpr vbn_step st = VBN_PLAN_STEPS[I];
  if constexpr (staged_kinds(KM)) {
    if constexpr (st.reserved[6] > 0) {
      step_barrier();
      constexpr int nxt = vbn_plan_next_mlp(I + 1);
      if constexpr (nxt >= 0) {
        vbn_plan_stage<nxt>(A, params, wbuf, par ^ 1, wave, nw, L.lane);
      } else {
        if (more) vbn_plan_stage<vbn_plan_next_mlp(0)>(A, params, wbuf, par ^ 1, wave, nw, L.lane);
      }
      L.wb = wbuf + par * A.wbuf_floats;
      par ^= 1;
    }
  } else {
    L.wb = params + st.reserved[5];
  }
  walk_step<KM>(A, st, L, lp);
}

template <unsigned KM, int... I>
__device__ __forceinline__ void vbn_plan_steps(const vbn_walk_args& A, const float* __restrict__ params, float* wbuf,
                                               int wave, int nw, Lane& L, float& lp, int& par, bool more,
                                               vbn_seq<int, I...>) {
  (vbn_plan_step<KM, I>(A, params, wbuf, wave, nw, L, lp, par, more), ...);
}

// lean walks: one pass, so every step's LDS buffer is known at compile time
template <unsigned KM, int I>
__device__ __forceinline__ void vbn_plan_step_lean(const vbn_walk_args& A, const float* __restrict__ params,
                                                   float* wbuf, int wave, int nw, Lane& L, float& lp) {
  constexpr vbn_step st = VBN_PLAN_STEPS[I];
  if constexpr (staged_kinds(KM)) {
    if constexpr (st.reserved[6] > 0) {
      step_barrier();
      constexpr int nxt = vbn_plan_next_mlp(I + 1);
      if constexpr (nxt >= 0) vbn_plan_stage<nxt>(A, params, wbuf, vbn_plan_parity(I) ^ 1, wave, nw, L.lane);
      L.wb = wbuf + vbn_plan_parity(I) * A.wbuf_floats;
    }
  } else {
    L.wb = params + st.reserved[5];
  }
  walk_step<KM>(A, st, L, lp);
}

template <unsigned KM, int... I>
__device__ __forceinline__ void vbn_plan_steps_lean(const vbn_walk_args& A, const float* __restrict__ params,
                                                    float* wbuf, int wave, int nw, Lane& L, float& lp,
                                                    vbn_seq<int, I...>) {
  (vbn_plan_step_lean<KM, I>(A, params, wbuf, wave, nw, L, lp), ...);
}


// vbn_walk_kernel (vbn_walk_impl.h) over the compile-time step table: the same prologue
// (segment-state resume), sweeps (Gibbs: A.gibbs_iters, else 1) and epilogue.  Kept as a copy
// rather than sharing a body with the interpreter: routing the interpreter through a shared
// body changed its register allocation (cfg3's lean set gained VGPR spills).
template <unsigned KM>
__device__ __forceinline__ void vbn_walk_plan_general(const vbn_walk_args& A, const float* __restrict__ params) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nw = blockDim.x >> 6, wave = threadIdx.x >> 6;
  const int per_wave = (A.n_slots + (A.max_out > 0 ? A.max_out : 1)) * WAVE;
  float* wbuf = smem + nw * per_wave;
  Lane L;
  L.P = params;
  L.ic = VBN_PLAN_IC;
  L.lane = threadIdx.x & (WAVE - 1);
  L.vals = smem + wave * per_wave;
  L.scr = L.vals + A.n_slots * WAVE;
  L.wb = wbuf;
  const int64_t total = A.n_queries * (int64_t)A.n_samples;
  L.mirror = (KM & 64) != 0;
  L.lean = (KM & 128) != 0;
  L.noiseless = (KM & (128 | 256)) != 0;
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
  if (!L.lean && A.state && (A.state_flags & 1)) {  // resume a segmented walk / the Gibbs start state
    for (int c = 0; c < A.n_slots; ++c) vwrite(L, c, A.state[(int64_t)c * total + L.p]);
    lp = A.state[(int64_t)A.n_slots * total + L.p];
    wave_sync();
  }
  const int iters = (!L.lean && A.mode == VBN_MODE_GIBBS) ? A.gibbs_iters : 1;
  int par = 0;
  if constexpr (staged_kinds(KM)) {
    constexpr int first = vbn_plan_next_mlp(0);
    if constexpr (first >= 0) vbn_plan_stage<first>(A, params, wbuf, 0, wave, nw, L.lane);
  }
  for (int it = 0; it < iters; ++it) {
    L.iter = it;
    // opaque per sweep: keeps the compiler from hoisting every step's parameter addresses,
    // parent-slot reads and Philox keys out of the sweep loop (83-step cfg2 sweep: 522 SGPR and
    // 361 VGPR spills without, 44 and 23 with)
    const float* P = params;
    const int32_t* IC = VBN_PLAN_IC;
    vbn_walk_args S = A;
    asm volatile("" : "+s"(P), "+s"(IC), "+s"(S.fixed), "+s"(S.noise), "+s"(S.seed), "+s"(S.offset),
                 "+s"(S.q_base), "+s"(S.out_x));
    L.P = P;
    L.ic = IC;
    vbn_plan_steps<KM>(S, P, wbuf, wave, nw, L, lp, par, it + 1 < iters,
                       __make_integer_seq<vbn_seq, int, VBN_PLAN_N_STEPS>{});
  }
  if (!valid || (L.mirror && L.lane >= 32)) return;
  if (A.mode == VBN_MODE_GIBBS) return;                  // outputs written by COLLECT steps
  if (!L.lean && A.state && (A.state_flags & 2)) {
    for (int c = 0; c < A.n_slots; ++c) A.state[(int64_t)c * total + L.p] = vread(L, c);
    A.state[(int64_t)A.n_slots * total + L.p] = lp;
  }
  if (A.out_lp && A.mode != VBN_MODE_SAMPLE) A.out_lp[L.p] = (A.mode == VBN_MODE_MCM) ? __expf(lp) : lp;
  if (A.out_x) {
    for (int k = 0; k < A.n_out_cols; ++k) A.out_x[L.p * A.n_out_cols + k] = vread(L, A.out_cols[k]);
  }
  if (A.stats_part && A.mode == VBN_MODE_MCM && L.wq && !L.mirror) stats_partials(A, L, __expf(lp));
}

// ------------------------------------------------------------------------------------------
// Gibbs sweeps on chain workgroups (VBN_PLAN_CHAIN_WAVES waves per workgroup, jit.py with a
// plan.gibbs_levels schedule).  A sweep at a few thousand chains leaves ~1 wave per SIMD, and
// that wave's serial path (83 dependent steps for the cfg2 DAG) is the bound, not issue.  Here
// the waves of a workgroup share ONE copy of their chains' slots in LDS and split each sweep's
// node updates between them: the updates of one level touch no slot another one writes, so
// they run at the same time on different waves, with one barrier per level (cfg2 DAG: 31
// serial steps instead of 83 on 4 waves).  Uneven levels run split (plan.gibbs_schedule): the
// LATENT steps, then every child step, then the SELECTs, a barrier after each phase, the scores
// passed through LDS rows (jit.py vbn_plan_step_lpout / _select) and added in sweep order.
// Every update runs the same device functions on the same values with the same draws (keyed by
// node, chain and sweep) as in the sequential sweep, so the chains are bit-identical to it.
// Weights come from the blob (L1/L2): the waves run different MLPs at once, so there is no
// per-workgroup staging.
#ifdef VBN_PLAN_CHAIN_WAVES
template <unsigned KM, int I>
__device__ __forceinline__ void vbn_plan_step_direct(const vbn_walk_args& A, const float* __restrict__ params,
                                                     Lane& L, float& lp) {
  constexpr vbn_step st = VBN_PLAN_STEPS[I];
  L.wb = params + st.reserved[5];
  walk_step<KM>(A, st, L, lp);
}

template <unsigned KM, int... I>
__device__ __forceinline__ void vbn_plan_run(const vbn_walk_args& A, const float* __restrict__ params, Lane& L,
                                             float& lp, vbn_seq<int, I...>) {
  (vbn_plan_step_direct<KM, I>(A, params, L, lp), ...);
}

// defined by the including unit (jit.py): every level's step ranges per wave, a barrier after each
template <unsigned KM>
__device__ __forceinline__ void vbn_plan_sweep_levels(const vbn_walk_args& A, const float* __restrict__ params,
                                                      int wave, Lane& L, float& lp);

template <unsigned KM>
__device__ __forceinline__ void vbn_walk_plan_chains(const vbn_walk_args& A, const float* __restrict__ params) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rows = A.max_out > 0 ? A.max_out : 1;
  Lane L;
  L.P = params;
  L.ic = VBN_PLAN_IC;
  L.lane = threadIdx.x & (WAVE - 1);
  L.vals = smem;                                       // the workgroup's chains, one copy
  L.scr = smem + A.n_slots * WAVE + wave * rows * WAVE;   // per-wave head / scratch rows
  L.wb = params;
  const int64_t total = A.n_queries * (int64_t)A.n_samples;
  L.mirror = (KM & 64) != 0;
  L.lean = false;
  L.noiseless = (KM & 256) != 0;
  L.bm_spare = 0.f;
  L.wq = false;
  const int wp = L.mirror ? 32 : WAVE;
  const int64_t p_raw = (int64_t)blockIdx.x * wp + (L.lane & (wp - 1));   // every wave: the same chains
  const bool valid = p_raw < total;
  L.p = valid ? p_raw : total - 1;
  L.b = L.p / A.n_samples;
  L.s = (int)(L.p - L.b * A.n_samples);
  L.iter = 0;
  L.valid = valid && wave == 0;                        // COLLECT: wave 0 writes the chains' outputs
  float lp = 0.f;
  if (A.state && (A.state_flags & 1)) {                // the start state (one ancestral pass)
    if (wave == 0)
      for (int c = 0; c < A.n_slots; ++c) vwrite(L, c, A.state[(int64_t)c * total + L.p]);
    lp = A.state[(int64_t)A.n_slots * total + L.p];
    __syncthreads();
  }
  for (int it = 0; it < A.gibbs_iters; ++it) {
    L.iter = it;
    const float* P = params;
    const int32_t* IC = VBN_PLAN_IC;
    vbn_walk_args S = A;
    asm volatile("" : "+s"(P), "+s"(IC), "+s"(S.fixed), "+s"(S.noise), "+s"(S.seed), "+s"(S.offset),
                 "+s"(S.q_base), "+s"(S.out_x));
    L.P = P;
    L.ic = IC;
    vbn_plan_sweep_levels<KM>(S, P, wave, L, lp);
  }
}
#endif

template <unsigned KM>
__device__ __forceinline__ void vbn_walk_plan_body(const vbn_walk_args& A, const float* __restrict__ params) {
  if constexpr ((KM & 128u) != 0) {      // lean (production MCM / IS / LW / ancestral): one pass
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int nw = blockDim.x >> 6, wave = threadIdx.x >> 6;
    const int per_wave = (A.n_slots + (A.max_out > 0 ? A.max_out : 1)) * WAVE;
    float* wbuf = smem + nw * per_wave;
    Lane L;
    L.P = params;
    L.ic = VBN_PLAN_IC;
    L.lane = threadIdx.x & (WAVE - 1);
    L.vals = smem + wave * per_wave;
    L.scr = L.vals + A.n_slots * WAVE;
    L.wb = wbuf;
    const int64_t total = A.n_queries * (int64_t)A.n_samples;
    L.mirror = false;
    L.lean = true;
    L.noiseless = true;
    L.bm_spare = 0.f;
    L.wq = (A.n_samples & (WAVE - 1)) == 0;
    const int64_t p_raw = ((int64_t)blockIdx.x * nw + wave) * WAVE + L.lane;
    const bool valid = p_raw < total;
    L.p = valid ? p_raw : total - 1;
    L.b = L.p / A.n_samples;
    L.s = (int)(L.p - L.b * A.n_samples);
    L.iter = 0;
    L.valid = valid;
    float lp = 0.f;
    if constexpr (staged_kinds(KM)) {
      constexpr int first = vbn_plan_next_mlp(0);
      if constexpr (first >= 0) vbn_plan_stage<first>(A, params, wbuf, 0, wave, nw, L.lane);
    }
    vbn_plan_steps_lean<KM>(A, params, wbuf, wave, nw, L, lp, __make_integer_seq<vbn_seq, int, VBN_PLAN_N_STEPS>{});
    if (!valid) return;
    if (A.out_lp && A.mode != VBN_MODE_SAMPLE) A.out_lp[L.p] = (A.mode == VBN_MODE_MCM) ? __expf(lp) : lp;
    if (A.out_x) {
      for (int k = 0; k < A.n_out_cols; ++k) A.out_x[L.p * A.n_out_cols + k] = vread(L, A.out_cols[k]);
    }
    if (A.stats_part && A.mode == VBN_MODE_MCM && L.wq) stats_partials(A, L, __expf(lp));
  } else {
#ifdef VBN_PLAN_CHAIN_WAVES
    vbn_walk_plan_chains<KM>(A, params);
#else
    vbn_walk_plan_general<KM>(A, params);
#endif
  }
}
