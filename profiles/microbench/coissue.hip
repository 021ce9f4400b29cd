// coissue.hip — does gfx950 overlap the KDE pass-1 instruction streams?  (MI355X)
//   hipcc -O3 --offload-arch=gfx950 profiles/microbench/coissue.hip -o /tmp/coissue && /tmp/coissue
// Kernels (every lane, `iters` trips, 256-thread blocks, 1/2/4 waves per SIMD):
//   exp      : 16 v_exp_f32 on independent chains per trip
//   add      : 16 v_add_f32 on independent chains per trip
//   exp_add  : both streams in one wave (independent)        -> exp + add co-issue?
//   mfma     : 4 v_mfma_f32_16x16x4_f32 per trip, independent accumulators
//   exp_mfma : 16 exps + 4 MFMAs per trip, independent        -> VALU / matrix-pipe overlap?
//   pass1    : the walk's pass-1 pattern, 4 MFMA tiles -> 16 exps on their results -> packed
//              sums (operands from registers)                 -> dependency cost
//   pass1_mem: pass1 with the point operand read from an L2-resident array
//   k32      : 32x32x2 pattern (2 MFMAs -> 32 exps -> 16 packed sums), operands from memory
// Prints per kernel the cycles per trip per SIMD (all waves of the SIMD together).
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
typedef float f32x2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) k_exp(float* out, const float* pts, int iters, float seed) {
  float x[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) x[c] = seed + 0.01f * (threadIdx.x + c);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = __builtin_amdgcn_exp2f(-x[c]);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_add(float* out, const float* pts, int iters, float seed) {
  float y[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) y[c] = seed * c;
  const float k = 1e-3f * seed;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 16; ++c) y[c] = y[c] + k;
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) s += y[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_exp_add(float* out, const float* pts, int iters, float seed) {
  float x[16], y[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) { x[c] = seed + 0.01f * (threadIdx.x + c); y[c] = seed * c; }
  const float k = 1e-3f * seed;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 16; ++c) { x[c] = __builtin_amdgcn_exp2f(-x[c]); y[c] = y[c] + k; }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) s += x[c] + y[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_mfma(float* out, const float* pts, int iters, float seed) {
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float a = seed * 0.01f, b = 0.02f * (threadIdx.x & 7);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_exp_mfma(float* out, const float* pts, int iters, float seed) {
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float x[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) x[c] = seed + 0.01f * (threadIdx.x + c);
  const float a = seed * 0.01f, b = 0.02f * (threadIdx.x & 7);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
#pragma unroll
      for (int c = 4 * t; c < 4 * t + 4; ++c) x[c] = __builtin_amdgcn_exp2f(-x[c]);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
#pragma unroll
  for (int c = 0; c < 16; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the walk's pass-1 trip for one block: 4 particle tiles, C = 0 (ZC form)
__device__ __forceinline__ void tile4(float a, const float (&b)[4], f32x2 (&acc)[4]) {
  f32x4 d[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) d[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[t], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    acc[t] += f32x2{__builtin_amdgcn_exp2f(d[t][0]), __builtin_amdgcn_exp2f(d[t][1])};
    acc[t] += f32x2{__builtin_amdgcn_exp2f(d[t][2]), __builtin_amdgcn_exp2f(d[t][3])};
  }
}

__global__ void __launch_bounds__(256) k_pass1(float* out, const float* pts, int iters, float seed) {
  const int lane = threadIdx.x & 63;
  float b[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) b[t] = (lane >> 4) == 3 ? -1.f : 0.01f * (lane + t) * seed;
  f32x2 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x2{0.f, 0.f};
  float a = -0.001f * lane;
  for (int i = 0; i < iters; ++i) {
    tile4(a, b, acc);
    a = -a;
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) s += acc[t].x + acc[t].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_pass1_mem(float* out, const float* pts, int iters, float seed) {
  const int lane = threadIdx.x & 63;
  float b[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) b[t] = (lane >> 4) == 3 ? -1.f : 0.01f * (lane + t) * seed;
  f32x2 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x2{0.f, 0.f};
  for (int i = 0; i < iters; i += 4) {
    float a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = pts[((i + u) & 1023) * 64 + lane];
#pragma unroll
    for (int u = 0; u < 4; ++u) tile4(a[u], b, acc);
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) s += acc[t].x + acc[t].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 32x32x2: one trip = 2 MFMAs (1024 pairs each) -> 32 exps -> 16 packed sums
__global__ void __launch_bounds__(256) k_k32(float* out, const float* pts, int iters, float seed) {
  const int lane = threadIdx.x & 63;
  const float bt0 = lane >= 32 ? -1.f : 0.02f * lane * seed, bt1 = lane >= 32 ? -1.f : 0.03f * lane * seed;
  f32x16 c0, c1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { c0[r] = -0.5f; c1[r] = -0.7f; }
  f32x2 acc0 = f32x2{0.f, 0.f}, acc1 = f32x2{0.f, 0.f};
  for (int i = 0; i < iters; ++i) {
    const float a = pts[(i & 1023) * 64 + lane];
    const f32x16 d0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bt0, c0, 0, 0, 0);
    const f32x16 d1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bt1, c1, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      acc0 += f32x2{__builtin_amdgcn_exp2f(d0[r]), __builtin_amdgcn_exp2f(d0[r + 1])};
      acc1 += f32x2{__builtin_amdgcn_exp2f(d1[r]), __builtin_amdgcn_exp2f(d1[r + 1])};
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc0.x + acc0.y + acc1.x + acc1.y;
}


// 16 exps + NP packed FMAs per trip, independent streams: do the packed FMAs issue under the
// exps' shadow?
template <int NP>
__global__ void __launch_bounds__(256) k_exp_pk(float* out, const float* pts, int iters, float seed) {
  float x[16];
  f32x2 y[NP];
#pragma unroll
  for (int c = 0; c < 16; ++c) x[c] = seed + 0.01f * (threadIdx.x + c);
#pragma unroll
  for (int c = 0; c < NP; ++c) y[c] = f32x2{seed * c, seed - c};
  const f32x2 a = {0.999f, 0.998f}, b = {1e-3f * seed, 2e-3f * seed};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      x[c] = __builtin_amdgcn_exp2f(-x[c]);
      if (c < NP) y[c] = __builtin_elementwise_fma(y[c], a, b);
      if (c + 16 < NP) y[c + 16] = __builtin_elementwise_fma(y[c + 16], a, b);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) s += x[c];
#pragma unroll
  for (int c = 0; c < NP; ++c) s += y[c].x + y[c].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// VALU pass 1 in the expanded form, points wave-uniform (scalar loads), two points per
// packed op: d = fma(y_0, 2x_0, -|x|^2) [+ fma(y_k, 2x_k, d)] - |y|^2; 16 points per trip
// (16 exps per lane).  Pack: [trip][NF + 1][16] floats.
template <int NF>
__global__ void __launch_bounds__(256) k_valu(float* out, const float* pts, int iters, float seed) {
  const int lane = threadIdx.x & 63;
  float xv[3];
  float nsq = 0.f;
#pragma unroll
  for (int f = 0; f < NF; ++f) { xv[f] = 0.01f * (lane + f) * seed; nsq = fmaf(xv[f], xv[f], nsq); }
  const f32x2 ns2 = {-nsq, -nsq};
  f32x2 acc = {0.f, 0.f}, acc2 = {0.f, 0.f};
  for (int i = 0; i < iters; ++i) {
    const float* __restrict__ p = pts + (i & 255) * (16 * (NF + 1));
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      f32x2 d = __builtin_elementwise_fma(f32x2{p[j], p[j + 1]}, f32x2{2.f * xv[0], 2.f * xv[0]}, ns2);
#pragma unroll
      for (int f = 1; f < NF; ++f)
        d = __builtin_elementwise_fma(f32x2{p[16 * f + j], p[16 * f + j + 1]}, f32x2{2.f * xv[f], 2.f * xv[f]}, d);
      d = d - f32x2{p[16 * NF + j], p[16 * NF + j + 1]};
      const f32x2 e = {__builtin_amdgcn_exp2f(d.x), __builtin_amdgcn_exp2f(d.y)};
      if (j & 2) acc2 += e; else acc += e;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x + acc.y + acc2.x + acc2.y;
}


// 16 v_fma_f32 (independent chains) + MF MFMAs per trip, independent streams: does the matrix
// pipe (f16 32x32x16 or f32 32x32x2) run under plain VALU work?
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <int KIND, int MF>
__global__ void __launch_bounds__(256) k_fma_mfma(float* out, const float* pts, int iters, float seed) {
  float x[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) x[c] = seed + 0.01f * (threadIdx.x + c);
  f32x16 acc[2];
  for (int c = 0; c < 2; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  f16x8 ah, bh;
  for (int r = 0; r < 8; ++r) { ah[r] = (_Float16)(seed * 0.01f * r); bh[r] = (_Float16)(0.02f * (threadIdx.x & 7)); }
  const float af = seed * 0.01f, bf = 0.02f * (threadIdx.x & 7);
  const float ka = 0.999f, kb = 1e-3f * seed;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int m = 0; m < MF; ++m) {
      if (KIND == 0) acc[m & 1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[m & 1], 0, 0, 0);
      else acc[m & 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(af, bf, acc[m & 1], 0, 0, 0);
#pragma unroll
      for (int c = (16 / MF) * m; c < (16 / MF) * (m + 1); ++c) x[c] = __builtin_fmaf(x[c], ka, kb);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) s += x[c];
  for (int r = 0; r < 16; ++r) s += acc[0][r] + acc[1][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int KIND, int MF>
__global__ void __launch_bounds__(256) k_mfma_only(float* out, const float* pts, int iters, float seed) {
  f32x16 acc[2];
  for (int c = 0; c < 2; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  f16x8 ah, bh;
  for (int r = 0; r < 8; ++r) { ah[r] = (_Float16)(seed * 0.01f * r); bh[r] = (_Float16)(0.02f * (threadIdx.x & 7)); }
  const float af = seed * 0.01f, bf = 0.02f * (threadIdx.x & 7);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int m = 0; m < MF; ++m) {
      if (KIND == 0) acc[m & 1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[m & 1], 0, 0, 0);
      else acc[m & 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(af, bf, acc[m & 1], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += acc[0][r] + acc[1][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_fma16(float* out, const float* pts, int iters, float seed) {
  float x[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) x[c] = seed + 0.01f * (threadIdx.x + c);
  const float ka = 0.999f, kb = 1e-3f * seed;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = __builtin_fmaf(x[c], ka, kb);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(float*, const float*, int, float);

static double run(kfn k, float* out, const float* pts, int blocks, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, pts, iters, 1.0f);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, pts, iters, 1.0f);
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
  float *out, *pts;
  CHECK(hipMalloc(&out, (size_t)ncu * 8 * 256 * sizeof(float)));
  CHECK(hipMalloc(&pts, 1024 * 64 * sizeof(float)));
  CHECK(hipMemset(pts, 0, 1024 * 64 * sizeof(float)));  // 256 KiB, L2-resident
  // exp_per_trip: v_exp_f32 wave instructions per trip (for the exp-issue fraction)
  struct { const char* name; kfn k; int iters; double exp_per_trip; } ks[] = {
      {"exp16", k_exp, 4096, 16},           {"add16", k_add, 4096, 0},
      {"exp16_add16", k_exp_add, 4096, 16}, {"mfma16x16x4_x4", k_mfma, 4096, 0},
      {"exp16_mfma16x16x4_x4", k_exp_mfma, 4096, 16},
      {"pass1_tile4_reg", k_pass1, 4096, 16}, {"pass1_tile4_mem", k_pass1_mem, 4096, 16},
      {"k32_2mfma_mem", k_k32, 4096, 32},
      {"exp16_pkfma8", k_exp_pk<8>, 4096, 16}, {"exp16_pkfma16", k_exp_pk<16>, 4096, 16},
      {"exp16_pkfma24", k_exp_pk<24>, 4096, 16}, 
      {"fma16", k_fma16, 4096, 0},
      {"mfma_f16_32x32x16_x2", k_mfma_only<0, 2>, 4096, 0}, {"fma16_mfma_f16_x2", k_fma_mfma<0, 2>, 4096, 0},
      {"mfma_f16_32x32x16_x4", k_mfma_only<0, 4>, 4096, 0}, {"fma16_mfma_f16_x4", k_fma_mfma<0, 4>, 4096, 0},
      {"mfma_f32_32x32x2_x2", k_mfma_only<1, 2>, 4096, 0}, {"fma16_mfma_f32_x2", k_fma_mfma<1, 2>, 4096, 0},
      {"valu_nf1", k_valu<1>, 4096, 16}, {"valu_nf2", k_valu<2>, 4096, 16}, {"valu_nf3", k_valu<3>, 4096, 16},
  };
  printf("{\"cus\": %d, \"clock_assumed_hz\": %.3g, \"results\": [\n", ncu, clk);
  bool first = true;
  for (auto& K : ks) {
    for (int wps = 1; wps <= 4; wps *= 2) {
      const int blocks = ncu * wps;
      const double t = run(K.k, out, pts, blocks, K.iters);
      const double cyc_trip = t * clk / ((double)wps * K.iters);   // per SIMD, all its waves
      const double frac = K.exp_per_trip > 0 ? K.exp_per_trip * 8.0 / cyc_trip : 0.0;
      printf("%s  {\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"simd_cycles_per_trip\": %.2f, \"wave_cycles_per_trip\": %.2f, "
             "\"exp_issue_frac\": %.3f}",
             first ? "" : ",\n", K.name, wps, t * 1e3, cyc_trip, cyc_trip * wps, frac);
      first = false;
    }
  }
  printf("\n]}\n");
  CHECK(hipFree(out));
  CHECK(hipFree(pts));
  return 0;
}
