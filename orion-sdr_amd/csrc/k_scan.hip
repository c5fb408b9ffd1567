// k_scan.hip — chunked state-carry scan kernels (see scan.hpp) for gfx950.
#include "scan.hpp"

namespace orion {
namespace {

constexpr int C = kScanC;
constexpr int NT = kScanNT;
constexpr int CH = kScanCH;
constexpr int PADN = CH + CH / 16 + 16;

__device__ __forceinline__ int pos(int e) { return e + (e >> 4); }

template <RecK RK> struct RecSel;
template <> struct RecSel<RecK::LP4> {
  using T = RecLP4;
  __device__ static T make(const ScanCoef& c) { return T{{c.b0, c.b1, c.b2, c.a1, c.a2}}; }
};
template <> struct RecSel<RecK::LPDC> {
  using T = RecLpDc;
  __device__ static T make(const ScanCoef& c) { return T{{c.b0, c.b1, c.b2, c.a1, c.a2}, c.r}; }
};
template <> struct RecSel<RecK::DC> {
  using T = RecDC;
  __device__ static T make(const ScanCoef& c) { return T{c.r}; }
};
template <> struct RecSel<RecK::ONEPOLE> {
  using T = RecOnePole;
  __device__ static T make(const ScanCoef& c) { return T{c.a}; }
};

// Translated (fm.rs:48-49) or raw complex sample i of channel ch; i may be the
// sample just before this workgroup. phasor(i) = e^{j theta (k0+i+1)}.
template <Pre PR>
__device__ __forceinline__ f2 cin(const ScanArgs& a, const f2* x, long long i, long long base, f2 Swg) {
  const f2 z = x[i];
  if constexpr (PR == Pre::Fm) {
    if (a.translate) {
      const f2 p = (i >= base) ? cmul(Swg, a.tab[i - base])
                               : phasor_q64(static_cast<uint64_t>(a.k0 + i + 1), a.step);
      const float c = p.x, d = -p.y;  // num-complex z * conj(p)
      return f2{z.x * c - z.y * d, z.x * d + z.y * c};
    }
  }
  return z;
}

// Pre-map of sample i (base <= i < n) -> recurrence input.
template <Pre PR>
__device__ __forceinline__ float premap(const ScanArgs& a, int ch, long long i, long long base, f2 Swg) {
  if constexpr (PR == Pre::Real) {
    return static_cast<const float*>(a.x)[ch * a.x_stride + i];
  } else {
    const f2* x = static_cast<const f2*>(a.x) + ch * a.x_stride;
    if constexpr (PR == Pre::Fm || PR == Pre::Pm) {
      const f2 z = cin<PR>(a, x, i, base, Swg);
      f2 p;
      if (i > 0) {
        p = cin<PR>(a, x, i - 1, base, Swg);
      } else {
        const float* cr = a.carry_in + ch * kScanCarry;
        p = f2{cr[6], cr[7]};
      }
      if constexpr (PR == Pre::Fm) return fm_disc(z, p, a.c.k);
      else return pm_disc(z, p, a.c.k);
    } else {
      const f2 z = x[i];
      if constexpr (PR == Pre::Ssb) {
        const f2 p = cmul(Swg, a.tab[i - base]);
        return __builtin_fmaf(z.x, p.x, z.y * p.y);  // ssb.rs:37
      } else if constexpr (PR == Pre::AmSqrt) {
        return __builtin_fmaf(z.x, z.x, z.y * z.y);  // am.rs:204
      } else if constexpr (PR == Pre::AmAbs) {
        return __builtin_fmaf(a.c.k1, fabsf(z.x), a.c.k2 * fabsf(z.y));  // am.rs:238
      } else {
        return sqrtf(z.x * z.x + z.y * z.y);  // cw.rs:38
      }
    }
  }
}

template <Pre PR>
__device__ __forceinline__ void stage(const ScanArgs& a, int ch, long long base, int cnt, float* sb) {
  f2 Swg = f2{1.0f, 0.0f};
  if constexpr (PR == Pre::Ssb || PR == Pre::Fm)
    Swg = phasor_q64(static_cast<uint64_t>(a.k0 + base + 1), a.step);
  for (int e = threadIdx.x; e < cnt; e += NT) sb[pos(e)] = premap<PR>(a, ch, base + e, base, Swg);
}

template <Post PO>
__device__ __forceinline__ float postmap(const ScanArgs& a, float y) {
  if constexpr (PO == Post::Sqrt) return sqrtf(y);  // am.rs:54 process_mapped(.., f32::sqrt)
  else if constexpr (PO == Post::Gain) return y * a.c.gain;  // cw.rs:41
  else return y;
}

template <RecK RK, Pre PR>
__global__ __launch_bounds__(NT) void k_scan_agg(const ScanArgs a) {
  using R = typename RecSel<RK>::T;
  constexpr int S = R::S;
  __shared__ float sb[PADN];
  __shared__ double tot[4][S];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int ch = blockIdx.y;
  const long long base = static_cast<long long>(blockIdx.x) * CH;
  const int cnt = static_cast<int>(min(static_cast<long long>(CH), a.n - base));
  const R rec = RecSel<RK>::make(a.c);
  stage<PR>(a, ch, base, cnt, sb);
  __syncthreads();
  float s[S];
#pragma unroll
  for (int i = 0; i < S; ++i) s[i] = 0.0f;
#pragma unroll
  for (int i = 0; i < C; ++i) {
    const int e = t * C + i;
    if (e < cnt) (void)rec.step(s, sb[pos(e)]);
  }
  double q[S];
#pragma unroll
  for (int i = 0; i < S; ++i) q[i] = s[i];
  wave_scan_inclusive<S>(q, a.mats + ScanMatsLayout::kPwc * S * S, lane);
  if (lane == 63)
#pragma unroll
    for (int i = 0; i < S; ++i) tot[wave][i] = q[i];
  __syncthreads();
  if (t == 0) {
    double g[S];
#pragma unroll
    for (int i = 0; i < S; ++i) g[i] = tot[0][i];
    for (int w = 1; w < 4; ++w) {
      double v[S];
#pragma unroll
      for (int i = 0; i < S; ++i) v[i] = tot[w][i];
      matvec_acc<S>(a.mats + ScanMatsLayout::kM64 * S * S, g, v);
#pragma unroll
      for (int i = 0; i < S; ++i) g[i] = v[i];
    }
    const long long nblk = gridDim.x;
    double* out = a.aggs + (ch * nblk + blockIdx.x) * S;
#pragma unroll
    for (int i = 0; i < S; ++i) out[i] = g[i];
  }
}

template <RecK RK>
__global__ __launch_bounds__(NT) void k_scan_carry(const ScanArgs a, int nblk) {
  constexpr int S = RecSel<RK>::T::S;
  __shared__ double q[2][NT][S];
  __shared__ double cs[S];
  const int t = threadIdx.x;
  const int ch = blockIdx.x;
  if (t < S) cs[t] = a.carry_in[ch * kScanCarry + t];
  __syncthreads();
  const double* Mch = a.mats + ScanMatsLayout::kPch * S * S;
  for (int c0 = 0; c0 < nblk; c0 += NT) {
    const int b = c0 + t;
    double v[S], carry[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
      carry[i] = cs[i];
      v[i] = b < nblk ? a.aggs[(static_cast<long long>(ch) * nblk + b) * S + i] : 0.0;
    }
    if (t == 0) matvec_acc<S>(Mch, carry, v);  // fold the incoming state into element 0
    int buf = 0;
    for (int s = 0; s < 8; ++s) {
      const int d = 1 << s;
#pragma unroll
      for (int i = 0; i < S; ++i) q[buf][t][i] = v[i];
      __syncthreads();
      if (t >= d) {
        double o[S];
#pragma unroll
        for (int i = 0; i < S; ++i) o[i] = q[buf][t - d][i];
        matvec_acc<S>(Mch + s * S * S, o, v);
      }
      buf ^= 1;
    }
#pragma unroll
    for (int i = 0; i < S; ++i) q[buf][t][i] = v[i];
    __syncthreads();
    if (b < nblk) {
      double* out = a.sin + (static_cast<long long>(ch) * nblk + b) * S;
#pragma unroll
      for (int i = 0; i < S; ++i) out[i] = t == 0 ? carry[i] : q[buf][t - 1][i];
    }
    __syncthreads();
    if (t < S) cs[t] = q[buf][NT - 1][t];
    __syncthreads();
  }
}

template <RecK RK, Pre PR, Post PO>
__global__ __launch_bounds__(NT) void k_scan_apply(const ScanArgs a) {
  using R = typename RecSel<RK>::T;
  constexpr int S = R::S;
  __shared__ float sb[PADN];
  __shared__ double tot[4][S];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int ch = blockIdx.y;
  const long long nblk = gridDim.x;
  const long long base = static_cast<long long>(blockIdx.x) * CH;
  const int cnt = static_cast<int>(min(static_cast<long long>(CH), a.n - base));
  const R rec = RecSel<RK>::make(a.c);
  stage<PR>(a, ch, base, cnt, sb);
  __syncthreads();
  float xs[C];
#pragma unroll
  for (int i = 0; i < C; ++i) xs[i] = sb[pos(t * C + i)];
  float s0[S];
#pragma unroll
  for (int i = 0; i < S; ++i) s0[i] = 0.0f;
#pragma unroll
  for (int i = 0; i < C; ++i)
    if (t * C + i < cnt) (void)rec.step(s0, xs[i]);
  double q[S];
#pragma unroll
  for (int i = 0; i < S; ++i) q[i] = s0[i];
  wave_scan_inclusive<S>(q, a.mats + ScanMatsLayout::kPwc * S * S, lane);
  if (lane == 63)
#pragma unroll
    for (int i = 0; i < S; ++i) tot[wave][i] = q[i];
  __syncthreads();
  // state entering this wave
  double cw[S];
  const double* sin = a.sin + (ch * nblk + blockIdx.x) * S;
#pragma unroll
  for (int i = 0; i < S; ++i) cw[i] = sin[i];
  for (int w = 0; w < wave; ++w) {
    double v[S];
#pragma unroll
    for (int i = 0; i < S; ++i) v[i] = tot[w][i];
    matvec_acc<S>(a.mats + ScanMatsLayout::kM64 * S * S, cw, v);
#pragma unroll
    for (int i = 0; i < S; ++i) cw[i] = v[i];
  }
  // state entering this lane: Q_{L-1} + A^{C L} cw
  double e[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const double o = __shfl_up(q[i], 1, 64);
    e[i] = lane == 0 ? 0.0 : o;
  }
  matvec_acc<S>(a.mats + (ScanMatsLayout::kLane + lane) * S * S, cw, e);
  float ef[S];
#pragma unroll
  for (int i = 0; i < S; ++i) ef[i] = static_cast<float>(e[i]);
  // re-run with the reference update
#pragma unroll
  for (int i = 0; i < C; ++i) {
    const int ei = t * C + i;
    if (ei < cnt) sb[pos(ei)] = postmap<PO>(a, rec.step(ef, xs[i]));
  }
  const bool last_blk = base + cnt == a.n;
  if (last_blk && t * C <= cnt - 1 && cnt - 1 < t * C + C) {
    float* co = a.carry_out + ch * kScanCarry;
    const float* ci = a.carry_in + ch * kScanCarry;
#pragma unroll
    for (int i = 0; i < S; ++i) co[i] = ef[i];
    for (int i = S; i < 6; ++i) co[i] = 0.0f;
    if constexpr (PR == Pre::Fm || PR == Pre::Pm) {
      const f2* x = static_cast<const f2*>(a.x) + ch * a.x_stride;
      f2 Swg = f2{1.0f, 0.0f};
      if constexpr (PR == Pre::Fm) Swg = phasor_q64(static_cast<uint64_t>(a.k0 + base + 1), a.step);
      const f2 z = cin<PR>(a, x, a.n - 1, base, Swg);
      co[6] = z.x;
      co[7] = z.y;
    } else {
      co[6] = ci[6];
      co[7] = ci[7];
    }
  }
  __syncthreads();
  float* y = static_cast<float*>(a.y) + ch * a.y_stride + base;
  for (int e2 = t; e2 < cnt; e2 += NT) y[e2] = sb[pos(e2)];
}

template <RecK RK, Pre PR, Post PO>
void run3(const ScanArgs& a, int nch, hipStream_t s) {
  const int nblk = div_up(a.n, CH);
  const dim3 grid(nblk, nch);
  k_scan_agg<RK, PR><<<grid, NT, 0, s>>>(a);
  k_scan_carry<RK><<<nch, NT, 0, s>>>(a, nblk);
  k_scan_apply<RK, PR, PO><<<grid, NT, 0, s>>>(a);
  ORION_LAUNCH_CHECK();
}

}  // namespace

int scan_state_dim(RecK rec) {
  switch (rec) {
    case RecK::LP4: return 4;
    case RecK::LPDC: return 6;
    case RecK::DC: return 2;
    default: return 1;
  }
}

void launch_scan(RecK rec, Pre pre, Post post, const ScanArgs& a, int nch, hipStream_t s) {
  if (a.n <= 0 || nch <= 0) return;
#define ORION_SCAN(RK, PR, PO) \
  if (rec == RecK::RK && pre == Pre::PR && post == Post::PO) return run3<RecK::RK, Pre::PR, Post::PO>(a, nch, s);
  ORION_SCAN(LP4, Real, Id)
  ORION_SCAN(DC, Real, Id)
  ORION_SCAN(LP4, Fm, Id)
  ORION_SCAN(LP4, Pm, Id)
  ORION_SCAN(LPDC, Ssb, Id)
  ORION_SCAN(LP4, AmSqrt, Sqrt)
  ORION_SCAN(LPDC, AmAbs, Id)
  ORION_SCAN(ONEPOLE, Cw, Gain)
#undef ORION_SCAN
  throw std::invalid_argument("unsupported scan combination");
}

}  // namespace orion
