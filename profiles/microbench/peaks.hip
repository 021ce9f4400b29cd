// peaks.hip — instruction-throughput microbenchmark for the roofline peaks bench.py prices
// the walk kernel against (MI355X / gfx950).  Build + run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 profiles/microbench/peaks.hip -o /tmp/peaks && /tmp/peaks
// Each kernel runs a grid of 256 CUs x W waves, every lane a few independent dependency
// chains of one instruction (negation / source modifiers only, so the chain is that
// instruction alone), and prints the chip-wide instruction rate and the implied cycles per
// wave64 instruction per SIMD at the clock given on the command line (default 2.4 GHz).
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
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define CH 8  // independent chains per lane

__global__ void __launch_bounds__(256) k_exp(float* out, int iters, float seed) {
  float x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = seed + 0.01f * (threadIdx.x + c);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = __builtin_amdgcn_exp2f(-x[c]);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_log(float* out, int iters, float seed) {
  float x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = seed + 1.5f + 0.01f * (threadIdx.x + c);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = __builtin_amdgcn_logf(__builtin_fabsf(x[c]));
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_fma(float* out, int iters, float seed) {
  float x[CH];
  const float a = 0.999f, b = 1e-3f * seed;
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = seed + 0.01f * (threadIdx.x + c);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = __builtin_fmaf(x[c], a, b);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_pkfma(float* out, int iters, float seed) {
  f32x2 x[CH];
  const f32x2 a = {0.999f, 0.998f}, b = {1e-3f * seed, 2e-3f * seed};
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = f32x2{seed + 0.01f * (threadIdx.x + c), seed - 0.01f * c};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = __builtin_elementwise_fma(x[c], a, b);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += x[c].x + x[c].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_mad64(float* out, int iters, float seed) {
  uint32_t x[CH], y[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) { x[c] = threadIdx.x * 7919u + c; y[c] = (uint32_t)seed + c; }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const uint64_t p = (uint64_t)0xD256D193u * x[c] + y[c];
      x[c] = (uint32_t)(p >> 32);
      y[c] = (uint32_t)p;
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= x[c] ^ y[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;
}

__global__ void __launch_bounds__(256) k_mfma_f16(float* out, int iters, float seed) {
  f32x16 acc[2];
  for (int c = 0; c < 2; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  f16x8 a, b;
  for (int r = 0; r < 8; ++r) { a[r] = (_Float16)(seed * 0.01f * r); b[r] = (_Float16)(0.02f * (threadIdx.x & 7)); }
  for (int i = 0; i < iters; ++i) {
    acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, acc[1], 0, 0, 0);
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += acc[0][r] + acc[1][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_mfma_f32(float* out, int iters, float seed) {
  f32x16 acc[2];
  for (int c = 0; c < 2; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  const float a = seed * 0.01f, b = 0.02f * (threadIdx.x & 7);
  for (int i = 0; i < iters; ++i) {
    acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, acc[1], 0, 0, 0);
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += acc[0][r] + acc[1][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(float*, int, float);

static double run(kfn k, float* out, int blocks, int threads, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0f);  // warm-up
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0f);
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

int main(int argc, char** argv) {
  const double clk = argc > 1 ? atof(argv[1]) : 2.4e9;
  int dev = 0, ncu = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int simds = ncu * 4;
  float* out;
  CHECK(hipMalloc(&out, (size_t)ncu * 8 * 256 * sizeof(float)));
  struct { const char* name; kfn k; int insts_per_iter; double flop_per_inst_lane; int mfma; } ks[] = {
      {"v_exp_f32", k_exp, CH, 0, 0},
      {"v_log_f32", k_log, CH, 0, 0},
      {"v_fma_f32", k_fma, CH, 2, 0},
      {"v_pk_fma_f32", k_pkfma, CH, 4, 0},
      {"v_mad_u64_u32", k_mad64, CH, 0, 0},
      {"mfma_32x32x16_f16", k_mfma_f16, 2, 0, 1},
      {"mfma_32x32x2_f32", k_mfma_f32, 2, 0, 2},
  };
  printf("{\"cus\": %d, \"clock_assumed_hz\": %.3g, \"results\": [\n", ncu, clk);
  const int iters = 4096;
  bool first = true;
  for (auto& K : ks) {
    for (int wps = 1; wps <= 8; wps *= 2) {             // waves per SIMD (256-thread blocks: 4 waves/CU each)
      const int blocks = ncu * wps;
      const double t = run(K.k, out, blocks, 256, iters);
      const double waves = (double)blocks * 4;
      const double wave_insts = waves * iters * K.insts_per_iter;
      const double cyc_per_inst = t * clk * simds / wave_insts;   // per wave64 instruction per SIMD
      double rate;
      const char* unit;
      if (K.mfma == 1) { rate = wave_insts * 32768.0 / t / 1e12; unit = "TFLOP/s"; }
      else if (K.mfma == 2) { rate = wave_insts * 4096.0 / t / 1e12; unit = "TFLOP/s"; }
      else if (K.flop_per_inst_lane > 0) { rate = wave_insts * 64 * K.flop_per_inst_lane / t / 1e12; unit = "TFLOP/s"; }
      else { rate = wave_insts * 64 / t / 1e12; unit = "T/s (lane ops)"; }
      printf("%s  {\"inst\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"rate\": %.3f, \"unit\": \"%s\", "
             "\"cycles_per_wave_inst_per_simd\": %.3f}",
             first ? "" : ",\n", K.name, wps, t * 1e3, rate, unit, cyc_per_inst);
      first = false;
    }
  }
  printf("\n]}\n");
  CHECK(hipFree(out));
  return 0;
}
