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
// and launches it through vbn_hip_walk_module (include/vbn_hip.h).  Lean full-wave walks only
// (no injected draws, no segment state, not Gibbs): the production MCM / IS / LW / ancestral path.
#include "vbn_walk_impl.h"

template <typename T, T... I>
struct vbn_seq {};

constexpr int vbn_plan_next_mlp(int j) {
  for (; j < VBN_PLAN_N_STEPS; ++j)
    if (VBN_PLAN_STEPS[j].reserved[6] > 0) return j;
  return -1;
}

// LDS weight buffer step i's block lives in: MLP steps alternate buffers 0, 1, 0, ...
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

template <unsigned KM, int I>
__device__ __forceinline__ void vbn_plan_step(const vbn_walk_args& A, const float* __restrict__ params, float* wbuf,
                                              int wave, int nw, Lane& L, float& lp) {
  constexpr vbn_step st = VBN_PLAN_STEPS[I];
  if constexpr (staged_kinds(KM)) {
    if constexpr (st.reserved[6] > 0) {          // MLP step: its block has landed, stage the next
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
__device__ __forceinline__ void vbn_plan_steps(const vbn_walk_args& A, const float* __restrict__ params, float* wbuf,
                                               int wave, int nw, Lane& L, float& lp, vbn_seq<int, I...>) {
  (vbn_plan_step<KM, I>(A, params, wbuf, wave, nw, L, lp), ...);
}

// The walk of vbn_walk_kernel (lean, full-wave form) over the compile-time step table.
template <unsigned KM>
__device__ __forceinline__ void vbn_walk_plan_body(const vbn_walk_args& A, const float* __restrict__ params) {
  static_assert((KM & 128u) != 0 && (KM & 64u) == 0, "plan-specialised walks are lean full-wave walks");
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
  vbn_plan_steps<KM>(A, params, wbuf, wave, nw, L, lp, __make_integer_seq<vbn_seq, int, VBN_PLAN_N_STEPS>{});
  if (!valid) return;
  if (A.out_lp && A.mode != VBN_MODE_SAMPLE) A.out_lp[L.p] = (A.mode == VBN_MODE_MCM) ? __expf(lp) : lp;
  if (A.out_x) {
    for (int k = 0; k < A.n_out_cols; ++k) A.out_x[L.p * A.n_out_cols + k] = vread(L, A.out_cols[k]);
  }
}
