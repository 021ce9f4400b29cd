// vbn_walk.hip — host entry points of the C-ABI (include/vbn_hip.h) and the small kernels
// (weight normalisation, RB epilogue, resampling, posterior statistics).  The walk kernel
// lives in vbn_walk_impl.h; its kind-set instantiations are compiled one per object from
// walk_inst.hip and launched through vbn_launch_walk_km<KM>.
#include "vbn_hip.h"
#include "vbn_walk_impl.h"

// the walk launchers, one per object compiled from walk_inst.hip
#define VBN_DECL(K) extern "C" hipError_t vbn_launch_walk_km##K(const vbn_walk_args*, dim3, dim3, size_t, hipStream_t);
VBN_WALK_KIND_SETS(VBN_DECL)
#undef VBN_DECL
// ------------------------------------------------------------------------------------------
// per-query weight normalisation (softmax over S + ESS, or max-shifted exp)
// ------------------------------------------------------------------------------------------
#define NW_THREADS 256

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// sqrt(var.clamp_min(0)) as torch computes it: clamp_min keeps a NaN (fmaxf would drop it)
__device__ __forceinline__ float std_of_var(float v) { return sqrtf(v < 0.f ? 0.f : v); }

// sum over the NW_THREADS threads of a workgroup (every thread gets the total)
__device__ __forceinline__ float nw_block_sum(float v, float* red) {
  v = wave_sum(v);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int k = 0; k < NW_THREADS / WAVE; ++k) t += red[k];
  return t;
}

// (ABI v13) the posterior summary fused into the normalisation (vbn_hip_normalize_weights_stats)
struct vbn_stats_out {
  const float* x;     // [B][S][dim] samples, or NULL: no summary
  float* mean;        // [B][dim]
  float* std;         // [B][dim]
  float* ess;         // [B]
  int dim;
  float eps;          // _posterior_stats' eps
};

// VBN._posterior_stats (vbn.py:495-503) of one row whose weights this thread holds in
// registers (pdf[j0 + k], k < PER): the same float arithmetic and reduction tree as
// vbn_posterior_stats_kernel, without reading the weights back.
template <int PER>
__device__ __forceinline__ void row_stats(const vbn_stats_out& so, const float (&pdf)[PER], int S, int j0,
                                          int64_t row, float* red) {
#pragma clang fp contract(off)
  float w[PER];
  float a = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const float v = pdf[k];
    w[k] = (j0 + k < S && !(v != v || v == INFINITY || v == -INFINITY)) ? fmaxf(v, 0.f) : 0.f;
    a += w[k];
  }
  const float denom = nw_block_sum(a, red);
  const bool ok = denom > so.eps;
  const float dn = fmaxf(denom, so.eps), uni = 1.0f / (float)max(1, S);
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (j0 + k < S) {
      w[k] = ok ? w[k] / dn : uni;
      q += w[k] * w[k];
    }
  }
  const float sq = nw_block_sum(q, red);
  if (threadIdx.x == 0) so.ess[row] = 1.0f / fmaxf(sq, so.eps);
  const int D = so.dim;
  const float* xr = so.x + row * (int64_t)S * D;
  for (int d = 0; d < D; ++d) {
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (j0 + k < S) m += w[k] * xr[(int64_t)(j0 + k) * D + d];
    const float mu = nw_block_sum(m, red);
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (j0 + k < S) {
        const float c = xr[(int64_t)(j0 + k) * D + d] - mu;
        v += w[k] * (c * c);
      }
    }
    const float var = nw_block_sum(v, red);
    if (threadIdx.x == 0) {
      so.mean[row * D + d] = mu;
      so.std[row * D + d] = std_of_var(var);
    }
  }
}

// run_if (ABI v11): when non-NULL and *run_if == 0 the launch writes nothing (the predicated
// fallback normalisation).  flag: when non-NULL, set to 1 (atomic OR) by every query whose
// ESS < ess_thr (a NaN ESS never sets it; importance_sampling.py:85-86); the caller zeroes it.
__global__ void __launch_bounds__(NW_THREADS) vbn_normalize_kernel(const float* log_w, float* w, float* ess,
                                                                  int S, int normalize, float eps,
                                                                  const int32_t* run_if, int32_t* flag,
                                                                  float ess_thr) {
  if (run_if && *run_if == 0) return;
  __shared__ float red[NW_THREADS / WAVE];
  __shared__ int nan_flag;
  const int64_t row = blockIdx.x;
  const float* x = log_w + row * S;
  float* y = w + row * S;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  if (tid == 0) nan_flag = 0;
  __syncthreads();
  float m = -INFINITY;
  int has_nan = 0;
  for (int i = tid; i < S; i += NW_THREADS) {
    const float v = x[i];
    has_nan |= (v != v);
    m = fmaxf(m, v);
  }
  if (has_nan) atomicOr(&nan_flag, 1);
  m = wave_max(m);
  if (lane == 0) red[wid] = m;
  __syncthreads();
  m = red[0];
  for (int k = 1; k < NW_THREADS / WAVE; ++k) m = fmaxf(m, red[k]);
  const bool row_nan = nan_flag != 0;
  __syncthreads();
  if (!normalize) {
    for (int i = tid; i < S; i += NW_THREADS) {
      const float v = expf(x[i] - m);                // all -inf row: exp(NaN) stays NaN
      y[i] = row_nan ? NAN : (v != v ? v : fmaxf(v, eps));
    }
    return;
  }
  float sum = 0.f;
  for (int i = tid; i < S; i += NW_THREADS) sum += expf(x[i] - m);
  sum = wave_sum(sum);
  if (lane == 0) red[wid] = sum;
  __syncthreads();
  sum = 0.f;
  for (int k = 0; k < NW_THREADS / WAVE; ++k) sum += red[k];
  __syncthreads();
  float sq = 0.f;
  for (int i = tid; i < S; i += NW_THREADS) {
    const float v = row_nan ? NAN : expf(x[i] - m) / sum;   // all -inf row: (-inf)-(-inf) -> NaN
    y[i] = v;
    sq += v * v;
  }
  sq = wave_sum(sq);
  if (lane == 0) red[wid] = sq;
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
    for (int k = 0; k < NW_THREADS / WAVE; ++k) t += red[k];
    const float e = 1.0f / t;
    if (ess) ess[row] = e;
    if (flag && e < ess_thr) atomicOr(flag, 1);
  }
}

// The same normalisation with the row held in registers (round 6): S <= NW_THREADS * PER, each
// thread keeps PER consecutive log-weights from ONE pass of 16-byte loads, and the max, the
// exp-sum and the normalised write + ESS all work on those registers -- one read of the row
// instead of three.  Reductions: per-thread partials over its PER values, then wave shuffles,
// then the 4 waves in LDS (the same tree as vbn_normalize_kernel; only each thread's share of
// the row is contiguous instead of strided).  cfg3: 14.0 us -> (r06b) per 4096 x 1024 call.
template <int PER>
__global__ void __launch_bounds__(NW_THREADS) vbn_normalize_reg_kernel(const float* __restrict__ log_w,
                                                                      float* __restrict__ w, float* __restrict__ ess,
                                                                      int S, int normalize, float eps,
                                                                      const int32_t* run_if, int32_t* flag,
                                                                      float ess_thr, const vbn_stats_out so) {
  if (run_if && *run_if == 0) return;
  __shared__ float red[NW_THREADS / WAVE];
  __shared__ int nan_flag;
  const int64_t row = blockIdx.x;
  const float* x = log_w + row * S;
  float* y = w + row * S;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int j0 = tid * PER;
  if (tid == 0) nan_flag = 0;
  float v[PER];
  const bool full = j0 + PER <= S && (S & 3) == 0;
  if (full) {
#pragma unroll
    for (int k = 0; k < PER; k += 4) {
      const float4 q = *reinterpret_cast<const float4*>(x + j0 + k);
      v[k] = q.x; v[k + 1] = q.y; v[k + 2] = q.z; v[k + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = j0 + k < S ? x[j0 + k] : -INFINITY;
  }
  float m = -INFINITY;
  int has_nan = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    has_nan |= (v[k] != v[k]);
    m = fmaxf(m, v[k]);
  }
  __syncthreads();                                   // nan_flag = 0 before any OR
  if (has_nan) atomicOr(&nan_flag, 1);
  m = wave_max(m);
  if (lane == 0) red[wid] = m;
  __syncthreads();
  m = red[0];
  for (int k = 1; k < NW_THREADS / WAVE; ++k) m = fmaxf(m, red[k]);
  const bool row_nan = nan_flag != 0;
  __syncthreads();
  float e[PER];
  if (!normalize) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      e[k] = 0.f;
      if (j0 + k < S) {
        const float t = expf(v[k] - m);               // all -inf row: exp(NaN) stays NaN
        e[k] = row_nan ? NAN : (t != t ? t : fmaxf(t, eps));
        y[j0 + k] = e[k];
      }
    }
    if (so.x) row_stats<PER>(so, e, S, j0, row, red);
    return;
  }
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    e[k] = j0 + k < S ? expf(v[k] - m) : 0.f;
    sum += e[k];
  }
  sum = wave_sum(sum);
  if (lane == 0) red[wid] = sum;
  __syncthreads();
  sum = 0.f;
  for (int k = 0; k < NW_THREADS / WAVE; ++k) sum += red[k];
  __syncthreads();
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const float q = row_nan ? NAN : e[k] / sum;      // all -inf row: (-inf)-(-inf) -> NaN
    e[k] = q;
    if (j0 + k < S) sq += q * q;
  }
  if (full) {
#pragma unroll
    for (int k = 0; k < PER; k += 4)
      *reinterpret_cast<float4*>(y + j0 + k) = make_float4(e[k], e[k + 1], e[k + 2], e[k + 3]);
  } else {
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (j0 + k < S) y[j0 + k] = e[k];
  }
  sq = wave_sum(sq);
  if (lane == 0) red[wid] = sq;
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
    for (int k = 0; k < NW_THREADS / WAVE; ++k) t += red[k];
    const float es = 1.0f / t;
    if (ess) ess[row] = es;
    if (flag && es < ess_thr) atomicOr(flag, 1);
  }
  if (so.x) row_stats<PER>(so, e, S, j0, row, red);
}

// ------------------------------------------------------------------------------------------
// multinomial resampling (resampled_importance_sampling.py:33-41): one 256-thread workgroup per
// query; inclusive CDF of the weights in LDS, one binary search per draw, state rows gathered
// slot-major (coalesced writes, reads within the query's row of particles).
// ------------------------------------------------------------------------------------------
#define RS_THREADS 256

__global__ void __launch_bounds__(RS_THREADS) vbn_resample_kernel(
    const float* __restrict__ w, const float* __restrict__ u, uint64_t seed, uint64_t offset, int64_t q_base,
    const float* __restrict__ sin, float* __restrict__ sout, int S, int n_cols, int64_t total) {
  extern __shared__ __attribute__((aligned(16))) float cdf[];
  __shared__ float seg[RS_THREADS];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const float* wr = w + b * S;
  // inclusive prefix sum: each thread a contiguous segment, then the segment totals
  const int per = (S + RS_THREADS - 1) / RS_THREADS;
  const int s0 = min(S, tid * per), s1 = min(S, s0 + per);
  float acc = 0.f;
  for (int s = s0; s < s1; ++s) { acc += wr[s]; cdf[s] = acc; }
  seg[tid] = acc;
  __syncthreads();
  if (tid == 0) {
    float run = 0.f;
    for (int k = 0; k < RS_THREADS; ++k) { const float v = seg[k]; seg[k] = run; run += v; }
  }
  __syncthreads();
  const float base = seg[tid];
  for (int s = s0; s < s1; ++s) cdf[s] += base;
  __syncthreads();
  const float tot = cdf[S - 1];
  for (int s = tid; s < S; s += RS_THREADS) {
    float uu;
    if (u) {
      uu = u[b * S + s];
    } else {
      const uint2 r = philox2x32(make_uint2((uint32_t)s, (uint32_t)(q_base + b + 1) ^ (uint32_t)(seed >> 32)),
                                 (uint32_t)seed + 0x7f000000u + (uint32_t)(offset & 0xffffffu));
      uu = u01(r.x);
    }
    const float thr = uu * tot;
    int lo = 0, hi = S - 1;                       // first k with cdf[k] > thr
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf[mid] > thr) hi = mid; else lo = mid + 1;
    }
    const int64_t src = b * S + lo, dst = b * S + s;
    for (int c = 0; c + 1 < n_cols; ++c) sout[(int64_t)c * total + dst] = sin[(int64_t)c * total + src];
    sout[(int64_t)(n_cols - 1) * total + dst] = 0.f;
  }
}

// ------------------------------------------------------------------------------------------
// Rao-Blackwellized epilogue (rao_blackwellized_marginalization.py:68-76, 255-317): one
// 256-thread workgroup per query; weights / component parameters staged in LDS, the mixture
// density evaluated with one grid point per thread (the component loop reads LDS broadcasts).
// ------------------------------------------------------------------------------------------
#define RB_THREADS 256

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int k = 0; k < RB_THREADS / WAVE; ++k) t += red[k];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = red[0];
  for (int k = 1; k < RB_THREADS / WAVE; ++k) t = fmaxf(t, red[k]);
  return t;
}

__global__ void __launch_bounds__(RB_THREADS) vbn_rb_epilogue_kernel(
    const float* __restrict__ log_w, const float* __restrict__ params, int64_t params_b,
    const float* __restrict__ z, float* __restrict__ pdf, float* __restrict__ grid, int P, int n_out,
    int mode, float stddevs, float min_scale, float eps) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ float red[RB_THREADS / WAVE];
  float* w = sm;            // [P]
  float* mu = sm + P;       // [P]   (gaussian)
  float* inv = sm + 2 * P;  // [P]   1/sigma
  float* cf = sm + 3 * P;   // [P]   w / (sqrt(2 pi) sigma)
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const float* lw = log_w + b * P;
  const float* prm = params + (params_b == 1 ? 0 : b) * (int64_t)P * (mode == 0 ? 2 : n_out);
  // _normalized_weights (68-76)
  float m = -INFINITY;
  for (int p = tid; p < P; p += RB_THREADS) {
    float v = lw[p];
    v = (v != v) ? -1e30f : (v == INFINITY ? 1e30f : (v == -INFINITY ? -1e30f : v));
    w[p] = v;
    m = fmaxf(m, v);
  }
  m = block_max(m, red);
  float s = 0.f;
  for (int p = tid; p < P; p += RB_THREADS) {
    const float e = expf(w[p] - m);
    w[p] = e;
    s += e;
  }
  const float denom = block_sum(s, red);
  const bool ok = denom > eps;
  const float dn = fmaxf(denom, eps), uni = 1.0f / (float)max(1, P);
  for (int p = tid; p < P; p += RB_THREADS) w[p] = ok ? w[p] / dn : uni;
  __syncthreads();
  if (mode == 1) {                                        // categorical (278)
    for (int c = 0; c < n_out; ++c) {
      float acc = 0.f;
      for (int p = tid; p < P; p += RB_THREADS) acc += w[p] * prm[(int64_t)p * n_out + c];
      const float t = block_sum(acc, red);
      if (tid == 0) pdf[b * n_out + c] = t;
    }
    return;
  }
  // gaussian mixture (297-317)
  float a1 = 0.f, a2 = 0.f;
  for (int p = tid; p < P; p += RB_THREADS) {
    const float loc = prm[2 * (int64_t)p];
    float sc = prm[2 * (int64_t)p + 1];
    sc = (sc != sc || sc == INFINITY || sc == -INFINITY) ? min_scale : fabsf(sc);
    sc = fmaxf(sc, min_scale);
    mu[p] = loc;
    inv[p] = 1.0f / sc;
    cf[p] = w[p] / (2.5066282746310002f * sc);
    a1 += w[p] * loc;
    a2 += w[p] * (sc * sc + loc * loc);
  }
  const float mean = block_sum(a1, red);
  const float second = block_sum(a2, red);
  const float var = fmaxf(second - mean * mean, min_scale * min_scale);
  const float sd = sqrtf(var);
  const float lo = mean - stddevs * sd, hi = mean + stddevs * sd;
  __syncthreads();
  for (int j = tid; j < n_out; j += RB_THREADS) {
    const float x = lo + (hi - lo) * z[j];
    float acc = 0.f;
    for (int p = 0; p < P; ++p) {
      const float zn = (x - mu[p]) * inv[p];
      acc = fmaf(cf[p], __expf(-0.5f * (zn * zn)), acc);
    }
    pdf[b * n_out + j] = acc;
    grid[b * n_out + j] = x;
  }
}

// ------------------------------------------------------------------------------------------
// weighted posterior summary (vbn.py:483-504): one 256-thread workgroup per query, two passes
// over the query's S particles (mean, then the centred second moment as the reference does).
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(RB_THREADS) vbn_posterior_stats_kernel(
    const float* __restrict__ pdf, const float* __restrict__ x, float* __restrict__ mean,
    float* __restrict__ stdv, float* __restrict__ ess, int S, int D, float eps) {
#pragma clang fp contract(off)
  __shared__ float red[RB_THREADS / WAVE];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const float* pr = pdf + b * S;
  const float* xr = x + b * (int64_t)S * D;
  auto wraw = [&](int s) {
    const float v = pr[s];
    return (v != v || v == INFINITY || v == -INFINITY) ? 0.f : fmaxf(v, 0.f);
  };
  float a = 0.f;
  for (int s = tid; s < S; s += RB_THREADS) a += wraw(s);
  const float denom = block_sum(a, red);
  const bool ok = denom > eps;
  const float dn = fmaxf(denom, eps), uni = 1.0f / (float)max(1, S);
  auto wt = [&](int s) { return ok ? wraw(s) / dn : uni; };
  float q = 0.f;
  for (int s = tid; s < S; s += RB_THREADS) {
    const float w = wt(s);
    q += w * w;
  }
  const float sq = block_sum(q, red);
  if (tid == 0) ess[b] = 1.0f / fmaxf(sq, eps);
  for (int d = 0; d < D; ++d) {
    float m = 0.f;
    for (int s = tid; s < S; s += RB_THREADS) m += wt(s) * xr[(int64_t)s * D + d];
    const float mu = block_sum(m, red);
    float v = 0.f;
    for (int s = tid; s < S; s += RB_THREADS) {
      const float c = xr[(int64_t)s * D + d] - mu;
      v += wt(s) * (c * c);
    }
    const float var = block_sum(v, red);
    if (tid == 0) {
      mean[b * D + d] = mu;
      stdv[b * D + d] = std_of_var(var);
    }
  }
}

// ------------------------------------------------------------------------------------------
// the same summary finished from the MCM walk's epilogue partials (vbn_walk_args.stats_part,
// vbn_walk_impl.h stats_partials): one thread per query merges its S / 64 wave rows in float64
// (Chan et al.'s pairwise update: M2 = sum_k M2_k + W_k (m_k - mean)^2).  Uniform weights where
// W <= eps (vbn.py:497-498): the unweighted (m_u, M2_u) rows, 64 particles each.
// ------------------------------------------------------------------------------------------
#define SM_THREADS 64
__global__ void __launch_bounds__(SM_THREADS) vbn_stats_merge_kernel(
    const double* __restrict__ part, int64_t n_queries, int n_parts, int D, float eps, float* __restrict__ mean,
    float* __restrict__ stdv, float* __restrict__ ess) {
  const int64_t b = (int64_t)blockIdx.x * SM_THREADS + threadIdx.x;
  if (b >= n_queries) return;
  const int stride = 2 + 4 * D;
  const double* r = part + b * n_parts * (int64_t)stride;
  double W = 0.0, Q = 0.0;
  for (int k = 0; k < n_parts; ++k) {
    W += r[(int64_t)k * stride];
    Q += r[(int64_t)k * stride + 1];
  }
  const bool ok = W > (double)eps;
  const double S = 64.0 * n_parts;
  if (ok) {
    ess[b] = 1.0f / fmaxf((float)(Q / (W * W)), eps);
  } else {
    const float uni = 1.0f / (float)max(1, 64 * n_parts);
    ess[b] = 1.0f / fmaxf((float)(64 * n_parts) * (uni * uni), eps);
  }
  for (int d = 0; d < D; ++d) {
    const int o = 2 + 4 * d + (ok ? 0 : 2);
    double m = 0.0;
    for (int k = 0; k < n_parts; ++k) {
      const double wk = ok ? r[(int64_t)k * stride] : 64.0;
      m += wk * r[(int64_t)k * stride + o];
    }
    m /= ok ? W : S;
    double m2 = 0.0;
    for (int k = 0; k < n_parts; ++k) {
      const double wk = ok ? r[(int64_t)k * stride] : 64.0;
      const double c = r[(int64_t)k * stride + o] - m;
      m2 += r[(int64_t)k * stride + o + 1] + wk * (c * c);   // 0 * NaN keeps a NaN sample's NaN
    }
    const double var = m2 / (ok ? W : S);
    mean[b * D + d] = (float)m;
    stdv[b * D + d] = std_of_var((float)var);
  }
}

// ------------------------------------------------------------------------------------------
// discrete weighted histogram of a target's samples (benchmarking/models/vbn.py:202-242,
// _estimate_discrete_posterior[_batch]): one lane per query walks its S (sample, weight) pairs
// in order -- the reference's float64 running sums, so the bins are bit-identical -- skipping
// non-finite weights and indices rint(x) outside [0, k); then _normalize_probs (vbn.py:116-121):
// total = numpy's pairwise sum of the bins (add.reduce from the identity 0.0), probs = bins /
// total, or 1/k each when total is not finite or <= 0.  A finite weight whose sample is NaN /
// +-inf is the reference's ValueError / OverflowError (int(round(x))): bad[b] records the first
// one (1 NaN, 2 inf) and the query's row is not meaningful.  Bins live in LDS ([k][64] doubles,
// k <= 128) or, for more bins, in the output row itself.
// ------------------------------------------------------------------------------------------
#define DP_THREADS 64
#define DP_LDS_BINS 128

// numpy pairwise_sum (umath loops_utils.h): n < 8 sequential from 0.0; n <= 128 eight strided
// accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus the tail; else split at
// n/2 rounded down to a multiple of 8.  D bounds the split depth at compile time (no recursion).
template <int D>
__device__ double np_pairwise_sum(const double* a, int64_t n, int64_t st) {
  if (n < 8) {
    double r = 0.0;
    for (int64_t i = 0; i < n; ++i) r += a[i * st];
    return r;
  }
  if (n <= 128 || D == 0) {
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = a[j * st];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] += a[(i + j) * st];
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i * st];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return np_pairwise_sum<(D > 0 ? D - 1 : 0)>(a, n2, st) + np_pairwise_sum<(D > 0 ? D - 1 : 0)>(a + n2 * st, n - n2, st);
}

// TX / TW: the samples' / weights' element type (float or double: the reference converts each
// with float(), so a float64 input bins and sums its own values, with no float32 rounding)
template <bool LDS_BINS, class TX, class TW>
__global__ void __launch_bounds__(DP_THREADS) vbn_discrete_posterior_kernel(
    const TX* __restrict__ x, int64_t x_stride, const TW* __restrict__ w, double* __restrict__ probs,
    int32_t* __restrict__ bad, int64_t B, int S, int k) {
#pragma clang fp contract(off)
  extern __shared__ double bins_lds[];
  const int64_t b = (int64_t)blockIdx.x * DP_THREADS + threadIdx.x;
  if (b >= B) return;                                    // no barriers below
  double* h = LDS_BINS ? bins_lds + threadIdx.x : probs + b * k;
  const int64_t hs = LDS_BINS ? DP_THREADS : 1;
  for (int c = 0; c < k; ++c) h[c * hs] = 0.0;
  const TX* xr = x + b * (int64_t)S * x_stride;
  const TW* wr = w + b * (int64_t)S;
  int flag = 0;
  for (int s = 0; s < S; ++s) {
    const TW wt = wr[s];
    if (!__builtin_isfinite(wt)) continue;
    const TX v = xr[(int64_t)s * x_stride];
    if (!__builtin_isfinite(v)) {
      flag = v != v ? 1 : 2;
      break;
    }
    const double r = __builtin_rint((double)v);        // round half to even, as Python's round
    if (r < 0.0 || r >= (double)k) continue;
    h[(int64_t)r * hs] += (double)wt;
  }
  bad[b] = flag;
  const double total = 0.0 + np_pairwise_sum<24>(h, k, hs);
  const bool ok = __builtin_isfinite(total) && total > 0.0;
  const double uni = 1.0 / (double)k;
  double* out = probs + b * k;
  for (int c = 0; c < k; ++c) out[c] = ok ? h[c * hs] / total : uni;
}

// ------------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------------
static thread_local char g_err[512];

static int fail(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

extern "C" int vbn_hip_abi_version(void) { return VBN_ABI_VERSION; }
extern "C" int vbn_hip_struct_size(int which) {
  return which == 0 ? (int)sizeof(vbn_walk_args) : (which == 1 ? (int)sizeof(vbn_step) : -1);
}
extern "C" const char* vbn_hip_last_error(void) { return g_err; }

extern "C" int64_t vbn_hip_lds_bytes(int32_t n_slots, int32_t max_out) {
  // the host sizes max_out >= KDE_CHUNKS when the plan walks a KDE node (chunk sums)
  return (int64_t)(n_slots + (max_out > 0 ? max_out : 1)) * WAVE * (int64_t)sizeof(float);
}

// Launch shape and instantiation of one walk: validates the arguments, picks the smallest
// instantiated kind set covering the plan and the workgroup size / LDS bytes (shared by the
// interpreter launch and the plan-specialised module launch).
struct walk_launch {
  unsigned kmi;      // instantiated kind set (VBN_WALK_KIND_SETS)
  dim3 grid, block;
  size_t lds;
};

static int walk_shape(const vbn_walk_args* a, walk_launch* out) {
  if (!a || (!a->steps && a->n_steps > 0) || a->n_steps < 0 || !a->params || a->n_samples <= 0 ||
      a->n_queries <= 0 || a->n_slots <= 0)
    return fail(VBN_E_ARGS, "vbn_hip_walk: bad arguments");
  if (a->out_x && (!a->out_cols || a->n_out_cols <= 0))
    return fail(VBN_E_ARGS, "vbn_hip_walk: out_x without out_cols");
  if ((a->state_flags & 4) && (!a->state || a->state_flags != 4 || a->noise || a->mode == VBN_MODE_GIBBS))
    return fail(VBN_E_ARGS, "vbn_hip_walk: state_flags 4 (precomputed per-sample quantities) needs a state "
                            "buffer and a walk without injected draws, segments or Gibbs sweeps");
  if (a->precomp_q && (a->noise || a->mode == VBN_MODE_GIBBS || (a->n_samples % WAVE) != 0 ||
                       a->wave_particles == 32 || (a->state && a->state_flags != 4)))
    return fail(VBN_E_ARGS, "vbn_hip_walk: precomp_q (per-query quantities) needs a lean full-wave walk "
                            "with n_samples a multiple of 64");
  if (a->stats_part && (a->mode != VBN_MODE_MCM || (a->n_samples % WAVE) != 0 || a->wave_particles == 32 ||
                        !a->out_cols || a->n_out_cols <= 0 || a->n_out_cols > 15))
    return fail(VBN_E_ARGS, "vbn_hip_walk: stats_part (fused posterior summary) needs an MCM full-wave walk "
                            "with n_samples a multiple of 64 and 1..15 output columns");
  if (a->wbuf_floats < 0 || (a->wbuf_floats % WBLK_CHUNK) != 0)
    return fail(VBN_E_ARGS, "vbn_hip_walk: wbuf_floats must be a non-negative multiple of 256");
  if (a->wave_particles != 0 && a->wave_particles != 32 && a->wave_particles != WAVE)
    return fail(VBN_E_ARGS, "vbn_hip_walk: wave_particles must be 0, 32 or 64");
  const int64_t wp = a->wave_particles == 32 ? 32 : WAVE;   // particles per wave
  // smallest instantiated kind set covering the plan (VBN_WALK_KIND_SETS)
  static const unsigned masks[] = {1u, 2u, 3u, 4u, 8u, 16u, 20u, 23u, 31u, 63u};
  const unsigned want = (unsigned)a->kind_mask & 63u;
  unsigned km = 63u;
  for (unsigned m : masks) {
    if ((m & want) == want && __builtin_popcount(m) < __builtin_popcount(km)) km = m;
  }
  const bool generic = ((unsigned)a->kind_mask & 512u) != 0;   // some MLP with other hidden_dims
  if (generic) km = 63u;
#ifdef VBN_KM_ONLY
  km = VBN_KM_ONLY & 63u;
#endif
  // waves per workgroup: staged kind sets take the most resident waves per CU (160 KiB LDS,
  // 16 waves = 4 per SIMD at the kernel's register budget), larger workgroups on ties (one
  // weight copy per workgroup); the other kind sets run one wave per workgroup
  const int64_t per_wave = vbn_hip_lds_bytes(a->n_slots, a->max_out);
  // small launches (e.g. Gibbs: one wave per 8 chains) keep >= 2 workgroups per CU first
  const int64_t waves = (a->n_queries * (int64_t)a->n_samples + wp - 1) / wp;
  int nw = 0;
  int64_t lds = 0;
  auto shape = [&](bool stg) {
    const int64_t wbuf_bytes = stg ? 2 * (int64_t)a->wbuf_floats * (int64_t)sizeof(float) : 0;
    int64_t best = 0;
    nw = 0;
    for (int w = stg ? WG_MAX_WAVES : 1; w >= 1; w >>= 1) {
      const int64_t l = w * per_wave + wbuf_bytes;
      if (l > 160 * 1024) continue;
      if (w > 1 && waves / w < 2 * 256) continue;
      const int64_t res = std::min<int64_t>(16, (160 * 1024 / l) * w);
      if (res > best) { best = res; nw = w; lds = l; }
    }
  };
  bool stage = staged_kinds(km);
  shape(stage);
#ifndef VBN_KM_ONLY
  if (stage && nw == 0) {
    // the two LDS weight buffers do not fit next to the value slots (very wide MLP fan-in):
    // run the smallest unstaged kind set covering the plan, which reads weights from the blob
    km = ((want & 32u) || generic) ? 63u : 23u;
    stage = false;
    shape(false);
  }
#endif
  if (nw == 0) return fail(VBN_E_LDS, "vbn_hip_walk: plan needs more than 160 KiB of LDS per wave");
  if (a->mode == VBN_MODE_GIBBS &&
      (a->n_samples != 8 || a->gibbs_iters <= 0 || a->gibbs_burn_in < 0 || a->gibbs_burn_in >= a->gibbs_iters ||
       a->gibbs_thin <= 0 || !a->out_x || (a->noise && a->n_noise <= 0)))
    return fail(VBN_E_ARGS, "vbn_hip_walk: Gibbs walk needs 8 candidates, iters > burn_in >= 0, thin > 0, out_x");
  const int64_t total = a->n_queries * (int64_t)a->n_samples;
  const int64_t blocks = (total + wp * nw - 1) / (wp * nw);
  if (blocks > 0x7fffffffLL) return fail(VBN_E_ARGS, "vbn_hip_walk: too many particles for one launch");
  // kind set | 64: the half-wave (mirror) instantiation; | 128: the lean one
  // lean: no injected draws, no segment state (state_flags 4 = read-only per-sample quantities
  // of VBN_F_PRECOMP steps, which the lean walk reads), not Gibbs
  const bool lean = !a->noise && (!a->state || a->state_flags == 4) && a->mode != VBN_MODE_GIBBS;
  out->kmi = km | (wp == 32 ? 64u : 0u) | (lean && wp != 32 ? 128u : 0u) |
             (wp == 32 && !a->noise ? 256u : 0u) |  // | 256: half-wave without injected draws
             (generic ? 512u : 0u);                 // | 512: with the generic-MLP path
  out->grid = dim3((unsigned)blocks);
  out->block = dim3(WAVE * nw);
  out->lds = (size_t)lds;
  return 0;
}

extern "C" int vbn_hip_walk_kind_set(const vbn_walk_args* a) {
  walk_launch w;
  const int rc = walk_shape(a, &w);
  return rc ? -rc : (int)w.kmi;
}

extern "C" int vbn_hip_walk(const vbn_walk_args* a, void* stream) {
  walk_launch w;
  const int rc = walk_shape(a, &w);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipErrorInvalidDeviceFunction;
#ifdef VBN_KM_ONLY
  // experiment builds (make exp KM=...): one instantiation only
  // (a lean-less set may serve a lean launch; never the reverse)
  const unsigned want = (unsigned)a->kind_mask & 63u;
  const bool lean = (w.kmi & 128u) != 0;
  const int64_t wp = a->wave_particles == 32 ? 32 : WAVE;
  if ((VBN_KM_ONLY & want) != want || ((VBN_KM_ONLY & 64) != 0) != (wp == 32) || ((VBN_KM_ONLY & 128) && !lean) ||
      ((VBN_KM_ONLY & 256) && a->noise))
    return fail(VBN_E_ARGS, "vbn_hip_walk: kind set not built in this experiment library");
  e = VBN_LAUNCHER(VBN_KM_ONLY)(a, w.grid, w.block, w.lds, st);
#else
  switch (w.kmi) {
#define VBN_CASE(K) case K##u: e = vbn_launch_walk_km##K(a, w.grid, w.block, w.lds, st); break;
    VBN_WALK_KIND_SETS(VBN_CASE)
#undef VBN_CASE
    default: break;
  }
#endif
  if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  return 0;
}

// ------------------------------------------------------------------------------------------
// plan-specialised walks: code objects compiled at run time (vbn_walk_plan.h)
// ------------------------------------------------------------------------------------------
struct vbn_plan_module {
  hipModule_t mod;
  hipFunction_t fn;
  unsigned kmi;
  int n_steps;
  int chain_waves;     // > 0: a Gibbs sweep on chain workgroups (vbn_hip_module_chain_waves)
  int static_lds;      // the kernel's static LDS (a sweep unit's vbn_lp_rows score rows), bytes
};

extern "C" int vbn_hip_module_load(const void* image, const char* kernel, uint32_t kind_set, int32_t n_steps,
                                   void** handle) {
  if (!image || !kernel || !handle) return fail(VBN_E_ARGS, "vbn_hip_module_load: bad arguments");
  vbn_plan_module* m = new vbn_plan_module{};
  hipError_t e = hipModuleLoadData(&m->mod, image);
  if (e == hipSuccess) e = hipModuleGetFunction(&m->fn, m->mod, kernel);
  if (e != hipSuccess) {
    if (m->mod) hipModuleUnload(m->mod);
    delete m;
    return fail((int)e, hipGetErrorString(e));
  }
  int st_lds = 0;
  if (hipFuncGetAttribute(&st_lds, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, m->fn) != hipSuccess) st_lds = 0;
  m->kmi = kind_set;
  m->n_steps = n_steps;
  m->static_lds = st_lds;
  *handle = m;
  return 0;
}

extern "C" int vbn_hip_module_unload(void* handle) {
  vbn_plan_module* m = (vbn_plan_module*)handle;
  if (!m) return 0;
  const hipError_t e = hipModuleUnload(m->mod);
  delete m;
  return e == hipSuccess ? 0 : fail((int)e, hipGetErrorString(e));
}

// chain workgroups run up to 8 waves (the jit.py sweep unit's launch bounds follow its wave count)
#define CHAIN_MAX_WAVES 8

extern "C" int vbn_hip_module_chain_waves(void* handle, int32_t n_waves) {
  vbn_plan_module* m = (vbn_plan_module*)handle;
  if (!m || n_waves < 1 || n_waves > CHAIN_MAX_WAVES)
    return fail(VBN_E_ARGS, "vbn_hip_module_chain_waves: bad module or wave count (1..8)");
  m->chain_waves = n_waves;
  return 0;
}

extern "C" int vbn_hip_walk_module(const void* handle, const vbn_walk_args* a, void* stream) {
  const vbn_plan_module* m = (const vbn_plan_module*)handle;
  if (!m) return fail(VBN_E_ARGS, "vbn_hip_walk_module: no module");
  walk_launch w;
  const int rc = walk_shape(a, &w);
  if (rc) return rc;
  // a Gibbs sweep without injected draws may run the draw-free (| 256) unit at full wave too:
  // the interpreter instantiates | 256 for half waves only, a plan unit is compiled per set
  // (full-wave cfg2 sweep: 97 VGPR spills with the injected-draw paths, none without)
  const unsigned free_km = w.kmi | ((a->mode == VBN_MODE_GIBBS && !a->noise) ? 256u : 0u);
  if ((m->kmi != w.kmi && m->kmi != free_km) || a->n_steps != m->n_steps)
    return fail(VBN_E_ARGS, "vbn_hip_walk_module: the launch does not match the compiled plan (kind set / steps)");
  if (m->chain_waves > 0) {
    // chain workgroups: every wave of a workgroup walks the same wp candidate lanes; one LDS
    // copy of their slots + per-wave scratch rows, no weight buffers
    if (a->mode != VBN_MODE_GIBBS)
      return fail(VBN_E_ARGS, "vbn_hip_walk_module: a chain-workgroup module runs Gibbs sweeps only");
    const int64_t wp = a->wave_particles == 32 ? 32 : WAVE;
    const int64_t rows = a->max_out > 0 ? a->max_out : 1;
    const int64_t lds = ((int64_t)a->n_slots + m->chain_waves * rows) * WAVE * (int64_t)sizeof(float);
    // the dynamic slots + scratch rows and the unit's static score rows share the CU's 160 KiB
    if (lds + m->static_lds > 160 * 1024)
      return fail(VBN_E_LDS, "vbn_hip_walk_module: chain workgroup needs more than 160 KiB of LDS");
    const int64_t blocks = (a->n_queries * (int64_t)a->n_samples + wp - 1) / wp;
    if (blocks > 0x7fffffffLL) return fail(VBN_E_ARGS, "vbn_hip_walk: too many particles for one launch");
    w.grid = dim3((unsigned)blocks);
    w.block = dim3(WAVE * m->chain_waves);
    w.lds = (size_t)lds;
  }
  vbn_walk_args args = *a;
  const float* params = a->params;
  void* kp[] = {&args, &params};
  const hipError_t e = hipModuleLaunchKernel(m->fn, w.grid.x, 1, 1, w.block.x, 1, 1, (unsigned)w.lds,
                                             (hipStream_t)stream, kp, nullptr);
  if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  return 0;
}

extern "C" int vbn_hip_posterior_stats(const float* pdf, const float* x, float* mean, float* std, float* ess,
                                       int64_t n_queries, int32_t n_samples, int32_t dim, float eps, void* stream) {
  if (!pdf || !x || !mean || !std || !ess || n_queries <= 0 || n_samples <= 0 || dim <= 0)
    return fail(VBN_E_ARGS, "vbn_hip_posterior_stats: bad arguments");
  hipLaunchKernelGGL(vbn_posterior_stats_kernel, dim3((unsigned)n_queries), dim3(RB_THREADS), 0,
                     (hipStream_t)stream, pdf, x, mean, std, ess, n_samples, dim, eps);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  return 0;
}

template <class TX, class TW>
static void launch_discrete_posterior(const void* x, int64_t x_stride, const void* w, double* probs, int32_t* bad,
                                      int64_t n_queries, int32_t n_samples, int32_t k, void* stream) {
  const unsigned grid = (unsigned)((n_queries + DP_THREADS - 1) / DP_THREADS);
  if (k <= DP_LDS_BINS)
    hipLaunchKernelGGL((vbn_discrete_posterior_kernel<true, TX, TW>), dim3(grid), dim3(DP_THREADS),
                       (size_t)k * DP_THREADS * sizeof(double), (hipStream_t)stream, (const TX*)x, x_stride,
                       (const TW*)w, probs, bad, n_queries, n_samples, k);
  else
    hipLaunchKernelGGL((vbn_discrete_posterior_kernel<false, TX, TW>), dim3(grid), dim3(DP_THREADS), 0,
                       (hipStream_t)stream, (const TX*)x, x_stride, (const TW*)w, probs, bad, n_queries, n_samples,
                       k);
}

extern "C" int vbn_hip_discrete_posterior_typed(const void* x, int32_t x_f64, int64_t x_stride, const void* w,
                                                int32_t w_f64, double* probs, int32_t* bad, int64_t n_queries,
                                                int32_t n_samples, int32_t k, void* stream) {
  if (!x || !w || !probs || !bad || x_stride <= 0 || n_queries <= 0 || n_samples <= 0 || k <= 0 ||
      (x_f64 != 0 && x_f64 != 1) || (w_f64 != 0 && w_f64 != 1))
    return fail(VBN_E_ARGS, "vbn_hip_discrete_posterior: bad arguments");
  if (x_f64 && w_f64)
    launch_discrete_posterior<double, double>(x, x_stride, w, probs, bad, n_queries, n_samples, k, stream);
  else if (x_f64)
    launch_discrete_posterior<double, float>(x, x_stride, w, probs, bad, n_queries, n_samples, k, stream);
  else if (w_f64)
    launch_discrete_posterior<float, double>(x, x_stride, w, probs, bad, n_queries, n_samples, k, stream);
  else
    launch_discrete_posterior<float, float>(x, x_stride, w, probs, bad, n_queries, n_samples, k, stream);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  return 0;
}

extern "C" int vbn_hip_discrete_posterior(const float* x, int64_t x_stride, const float* w, double* probs,
                                          int32_t* bad, int64_t n_queries, int32_t n_samples, int32_t k,
                                          void* stream) {
  return vbn_hip_discrete_posterior_typed(x, 0, x_stride, w, 0, probs, bad, n_queries, n_samples, k, stream);
}

extern "C" int vbn_hip_resample(const float* w, const float* u, uint64_t seed, uint64_t offset, int64_t q_base,
                                const float* state_in, float* state_out, int64_t n_queries, int32_t n_samples,
                                int32_t n_cols, void* stream) {
  if (!w || !state_in || !state_out || state_in == state_out || n_queries <= 0 || n_samples <= 0 || n_cols <= 0)
    return fail(VBN_E_ARGS, "vbn_hip_resample: bad arguments");
  const size_t lds = (size_t)n_samples * sizeof(float);
  if (lds > 64 * 1024) return fail(VBN_E_LDS, "vbn_hip_resample: more than 16384 samples per query");
  hipLaunchKernelGGL(vbn_resample_kernel, dim3((unsigned)n_queries), dim3(RS_THREADS), lds, (hipStream_t)stream,
                     w, u, seed, offset, q_base, state_in, state_out, n_samples, n_cols,
                     n_queries * (int64_t)n_samples);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  return 0;
}

extern "C" int vbn_hip_rb_epilogue(const float* log_w, const float* params, int64_t params_b, const float* z,
                                   float* pdf, float* grid, int64_t n_queries, int32_t n_particles, int32_t n_out,
                                   int32_t mode, float stddevs, float min_scale, float eps, void* stream) {
  if (!log_w || !params || !pdf || n_queries <= 0 || n_particles <= 0 || n_out <= 0 || (mode != 0 && mode != 1) ||
      (mode == 0 && (!z || !grid)) || (params_b != 1 && params_b != n_queries))
    return fail(VBN_E_ARGS, "vbn_hip_rb_epilogue: bad arguments");
  const size_t lds = (size_t)n_particles * 4 * sizeof(float);
  if (lds > 64 * 1024) return fail(VBN_E_LDS, "vbn_hip_rb_epilogue: more than 4096 particles per query");
  hipLaunchKernelGGL(vbn_rb_epilogue_kernel, dim3((unsigned)n_queries), dim3(RB_THREADS), lds,
                     (hipStream_t)stream, log_w, params, params_b, z, pdf, grid, n_particles, n_out, mode,
                     stddevs, min_scale, eps);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  return 0;
}

static int normalize_launch(const float* log_w, float* w, float* ess, int64_t n_queries, int32_t n_samples,
                            int32_t normalize, float eps, const int32_t* run_if, int32_t* flag, float ess_thr,
                            const vbn_stats_out& so, void* stream) {
  if (!log_w || !w || n_queries <= 0 || n_samples <= 0 || (flag && !normalize))
    return fail(VBN_E_ARGS, "vbn_hip_normalize_weights: bad arguments");
  // rows of up to 4096 weights stay in registers (vbn_normalize_reg_kernel; 16-byte loads need
  // 16-byte aligned rows); longer rows stream three times through the strided form
  const bool al = ((uintptr_t)log_w & 15) == 0 && ((uintptr_t)w & 15) == 0;
  if (so.x && !(al && n_samples <= NW_THREADS * 16))
    return fail(VBN_E_ARGS, "vbn_hip_normalize_weights_stats: needs n_samples <= 4096 and 16-byte aligned rows");
  const dim3 g((unsigned)n_queries), blk(NW_THREADS);
  hipStream_t st = (hipStream_t)stream;
  if (al && n_samples <= NW_THREADS * 4)
    hipLaunchKernelGGL(vbn_normalize_reg_kernel<4>, g, blk, 0, st, log_w, w, ess, n_samples, normalize, eps, run_if,
                       flag, ess_thr, so);
  else if (al && n_samples <= NW_THREADS * 8)
    hipLaunchKernelGGL(vbn_normalize_reg_kernel<8>, g, blk, 0, st, log_w, w, ess, n_samples, normalize, eps, run_if,
                       flag, ess_thr, so);
  else if (al && n_samples <= NW_THREADS * 16)
    hipLaunchKernelGGL(vbn_normalize_reg_kernel<16>, g, blk, 0, st, log_w, w, ess, n_samples, normalize, eps, run_if,
                       flag, ess_thr, so);
  else
    hipLaunchKernelGGL(vbn_normalize_kernel, g, blk, 0, st, log_w, w, ess, n_samples, normalize, eps, run_if, flag,
                       ess_thr);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  return 0;
}

extern "C" int vbn_hip_normalize_weights_ex(const float* log_w, float* w, float* ess, int64_t n_queries,
                                            int32_t n_samples, int32_t normalize, float eps, const int32_t* run_if,
                                            int32_t* flag, float ess_thr, void* stream) {
  const vbn_stats_out none{nullptr, nullptr, nullptr, nullptr, 0, 0.f};
  return normalize_launch(log_w, w, ess, n_queries, n_samples, normalize, eps, run_if, flag, ess_thr, none, stream);
}

extern "C" int vbn_hip_normalize_weights_stats(const float* log_w, float* w, float* ess, int64_t n_queries,
                                               int32_t n_samples, int32_t normalize, float eps,
                                               const int32_t* run_if, int32_t* flag, float ess_thr, const float* x,
                                               int32_t dim, float stats_eps, float* mean, float* std,
                                               float* stats_ess, void* stream) {
  if (!x || !mean || !std || !stats_ess || dim <= 0)
    return fail(VBN_E_ARGS, "vbn_hip_normalize_weights_stats: bad arguments");
  const vbn_stats_out so{x, mean, std, stats_ess, dim, stats_eps};
  return normalize_launch(log_w, w, ess, n_queries, n_samples, normalize, eps, run_if, flag, ess_thr, so, stream);
}

extern "C" int vbn_hip_posterior_stats_merge(const double* part, int64_t n_queries, int32_t n_parts, int32_t dim,
                                             float eps, float* mean, float* std, float* ess, void* stream) {
  if (!part || !mean || !std || !ess || n_queries <= 0 || n_parts <= 0 || dim <= 0 || dim > 15)
    return fail(VBN_E_ARGS, "vbn_hip_posterior_stats_merge: bad arguments");
  const int64_t blocks = (n_queries + SM_THREADS - 1) / SM_THREADS;
  hipLaunchKernelGGL(vbn_stats_merge_kernel, dim3((unsigned)blocks), dim3(SM_THREADS), 0, (hipStream_t)stream, part,
                     n_queries, n_parts, dim, eps, mean, std, ess);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  return 0;
}

extern "C" int vbn_hip_normalize_weights(const float* log_w, float* w, float* ess, int64_t n_queries,
                                         int32_t n_samples, int32_t normalize, float eps, void* stream) {
  return vbn_hip_normalize_weights_ex(log_w, w, ess, n_queries, n_samples, normalize, eps, nullptr, nullptr, 0.f,
                                      stream);
}
