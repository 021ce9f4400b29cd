// coissue_sgb.hip — MFMA / VALU co-issue with hand-placed fillers (MI355X, gfx950).
//   hipcc -O3 --offload-arch=gfx950 profiles/microbench/coissue_sgb.hip -o /tmp/coissue_sgb && /tmp/coissue_sgb
// One wave per SIMD (one 256-thread block per CU) unless stated.  Per trip: NM MFMAs, each
// followed by exactly K independent v_fma_f32 fillers, the order pinned with
// __builtin_amdgcn_sched_group_barrier (mask 0x008 = MFMA, 0x002 = VALU), so the fillers sit in
// the MFMA gaps instead of being clumped by the scheduler.  Variants:
//   f16_ind  : v_mfma_f32_32x32x16_f16, 4 independent accumulators (the walk's layer 2, two groups x 2)
//   f16_dep  : the same MFMA on ONE accumulator (dependent chain, as one group's K accumulation)
//   f32_ind  : v_mfma_f32_32x32x2_f32, 4 independent accumulators (the walk's layer 1)
// K = 0 gives the bare MFMA time; "fma_only" the fillers alone.  The guide
// (MI355X_MICROARCH.md, vector-instruction issue cost) expects a 32x32x16 gap to absorb
// fillers whose issue costs sum to <= 24 cycles (~6 v_fma_f32) nearly for free.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// KIND 0: f16 independent, 1: f16 dependent, 2: f32 independent, 3: fillers only
template <int KIND, int K>
__global__ void __launch_bounds__(256) k_sgb(float* out, int iters, float seed) {
  constexpr int NM = 8;
  constexpr int NF = K > 0 ? K * NM : 1;
  float x[NF];
#pragma unroll
  for (int c = 0; c < NF; ++c) x[c] = seed + 0.01f * (threadIdx.x + c);
  f32x16 acc[4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
  f16x8 ah, bh;
#pragma unroll
  for (int r = 0; r < 8; ++r) { ah[r] = (_Float16)(seed * 0.01f * r); bh[r] = (_Float16)(0.02f * (threadIdx.x & 7)); }
  const float af = seed * 0.01f, bf = 0.02f * (threadIdx.x & 7);
  const float ka = 0.999f, kb = 1e-3f * seed;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      const int a = KIND == 1 ? 0 : (m & 3);
      if constexpr (KIND == 0 || KIND == 1) acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[a], 0, 0, 0);
      else if constexpr (KIND == 2) acc[a] = __builtin_amdgcn_mfma_f32_32x32x2f32(af, bf, acc[a], 0, 0, 0);
#pragma unroll
      for (int c = 0; c < K; ++c) x[m * K + c] = __builtin_fmaf(x[m * K + c], ka, kb);
      if constexpr (KIND != 3) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if constexpr (K > 0) __builtin_amdgcn_sched_group_barrier(0x002, K, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NF; ++c) s += x[c];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[a][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(float*, int, float);

static double run(kfn k, float* out, int blocks, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return best * 1e-3;
}

#define ROW(KIND, K, NAME) {NAME, KIND, K, k_sgb<KIND, K>}

int main(int argc, char** argv) {
  const double clk = argc > 1 ? atof(argv[1]) : 2.4e9;
  int dev = 0, ncu = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  float* out;
  CHECK(hipMalloc(&out, (size_t)ncu * 4 * 256 * sizeof(float)));
  struct { const char* name; int kind, k; kfn f; } ks[] = {
      ROW(0, 0, "f16_ind"), ROW(0, 2, "f16_ind"), ROW(0, 4, "f16_ind"), ROW(0, 6, "f16_ind"), ROW(0, 8, "f16_ind"),
      ROW(0, 12, "f16_ind"),
      ROW(1, 0, "f16_dep"), ROW(1, 2, "f16_dep"), ROW(1, 4, "f16_dep"), ROW(1, 6, "f16_dep"), ROW(1, 8, "f16_dep"),
      ROW(2, 0, "f32_ind"), ROW(2, 2, "f32_ind"), ROW(2, 4, "f32_ind"), ROW(2, 8, "f32_ind"), ROW(2, 16, "f32_ind"),
      ROW(3, 2, "fma_only"), ROW(3, 4, "fma_only"), ROW(3, 6, "fma_only"), ROW(3, 8, "fma_only"), ROW(3, 16, "fma_only"),
  };
  const int iters = 2048;
  printf("{\"cus\": %d, \"clock_assumed_hz\": %.3g, \"mfma_per_trip\": 8, \"results\": [\n", ncu, clk);
  bool first = true;
  for (auto& K : ks) {
    for (int wps = 1; wps <= 2; ++wps) {
      const double t = run(K.f, out, ncu * wps, iters);
      const double cyc = t * clk / ((double)wps * iters * 8);   // SIMD cycles per MFMA slot (all waves)
      printf("%s  {\"kernel\": \"%s\", \"fillers_per_mfma\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, "
             "\"simd_cycles_per_mfma\": %.2f}", first ? "" : ",\n", K.name, K.k, wps, t * 1e3, cyc);
      first = false;
    }
  }
  printf("\n]}\n");
  CHECK(hipFree(out));
  return 0;
}
