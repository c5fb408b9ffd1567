// k_scan.hip — chunked state-carry scan kernels (see scan.hpp) for gfx950.
#include <cstdlib>
#include <type_traits>

#include "scan.hpp"

namespace orion {
namespace {

constexpr int C = kScanC;
constexpr int NT = kScanNT;
constexpr int CH = kScanCH;
constexpr int PADN = CH + CH / 16 + 16;
// Tuning constants (each measured A/B; HISTORY.md):
constexpr int kSpMinW = 4;       // waves per SIMD k_lpdc_sp is compiled for at kSpC samples per lane (<= 128 VGPRs)
constexpr int kSpMinW16 = 6;     // the same at 16 samples per lane
constexpr int kSpBatch = 8;      // k_scan_sp staging: loads issued together per thread (complex input)
constexpr int kSpBatchReal = 8;  // (real input)
constexpr int kScanSpMinW = 4;   // waves per SIMD k_scan_sp is compiled for (4: <= 128 VGPRs, spills 52-132 B)

__device__ __forceinline__ int pos(int e) { return e + (e >> 4); }

template <RecK RK> struct RecSel;
template <> struct RecSel<RecK::LP4> {
  using T = RecLP4;
  __device__ static T make(const ScanCoef& c) { return T{{c.b0, c.b1, c.b2, c.a1, c.a2}}; }
};
template <> struct RecSel<RecK::BQ> {
  using T = RecBQ;
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
// sample just before this workgroup. Sample i's phasor: oscillator output k0 + i (R:
// the cursor of the workgroup's run from sample base).
template <Pre PR>
__device__ __forceinline__ f2 cin(const ScanArgs& a, const f2* x, long long i, long long base, const OscRun& R) {
  const f2 z = x[i];
  if constexpr (PR == Pre::Fm) {
    if (a.translate) {
      const f2 p = (i >= base) ? osc_get(a.osc, R, static_cast<int>(i - base))
                               : osc_at(a.osc, static_cast<uint64_t>(a.k0 + i));
      const float c = p.x, d = -p.y;  // num-complex z * conj(p)
      return f2{z.x * c - z.y * d, z.x * d + z.y * c};
    }
  }
  return z;
}

// Pre-map of sample i (base <= i < n) -> recurrence input.
template <Pre PR>
__device__ __forceinline__ float premap(const ScanArgs& a, int ch, long long i, long long base, const OscRun& R) {
  if constexpr (PR == Pre::Real) {
    return static_cast<const float*>(a.x)[ch * a.x_stride + i];
  } else {
    const f2* x = static_cast<const f2*>(a.x) + ch * a.x_stride;
    if constexpr (PR == Pre::Fm || PR == Pre::Pm) {
      const f2 z = cin<PR>(a, x, i, base, R);
      f2 p;
      if (i > 0) {
        p = cin<PR>(a, x, i - 1, base, R);
      } else {
        const float* cr = a.carry_in + ch * kScanCarry;
        p = f2{cr[6], cr[7]};
      }
      if constexpr (PR == Pre::Fm) return fm_disc(z, p, a.c.k);
      else return pm_disc(z, p, a.c.k);
    } else {
      const f2 z = x[i];
      if constexpr (PR == Pre::Ssb) {
        const f2 p = osc_get(a.osc, R, static_cast<int>(i - base));
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

// premap with the samples already loaded: z = x[i], zp = x[i - 1] (any value when
// i == 0: the carried previous sample is used), raw (untranslated) complex samples.
template <Pre PR>
__device__ __forceinline__ f2 cin_v(const ScanArgs& a, f2 z, long long i, long long base, const OscRun& R) {
  if constexpr (PR == Pre::Fm) {
    if (a.translate) {
      const f2 p = (i >= base) ? osc_get(a.osc, R, static_cast<int>(i - base))
                               : osc_at(a.osc, static_cast<uint64_t>(a.k0 + i));
      const float c = p.x, d = -p.y;  // num-complex z * conj(p)
      return f2{z.x * c - z.y * d, z.x * d + z.y * c};
    }
  }
  return z;
}
template <Pre PR>
__device__ __forceinline__ float premap_v(const ScanArgs& a, int ch, long long i, long long base, const OscRun& R,
                                          f2 z, f2 zp) {
  if constexpr (PR == Pre::Fm || PR == Pre::Pm) {
    const f2 zc = cin_v<PR>(a, z, i, base, R);
    f2 p;
    if (i > 0) {
      p = cin_v<PR>(a, zp, i - 1, base, R);
    } else {
      const float* cr = a.carry_in + ch * kScanCarry;
      p = f2{cr[6], cr[7]};
    }
    if constexpr (PR == Pre::Fm) return fm_disc(zc, p, a.c.k);
    else return pm_disc(zc, p, a.c.k);
  } else if constexpr (PR == Pre::AmSqrt) {
    return __builtin_fmaf(z.x, z.x, z.y * z.y);  // am.rs:204
  } else if constexpr (PR == Pre::Cw) {
    return sqrtf(z.x * z.x + z.y * z.y);  // cw.rs:38
  } else {
    return z.x;  // Pre::Real: the f32 sample in z.x
  }
}

template <Pre PR>
__device__ __forceinline__ void stage(const ScanArgs& a, int ch, long long base, int cnt, float* sb) {
  OscRun R{};
  if constexpr (PR == Pre::Ssb || PR == Pre::Fm)
    if (PR == Pre::Ssb || a.translate) R = osc_run(a.osc, static_cast<uint64_t>(a.k0 + base), cnt);
  if constexpr (PR == Pre::Fm || PR == Pre::Pm) {
    for (int e = threadIdx.x; e < cnt; e += NT) sb[pos(e)] = premap<PR>(a, ch, base + e, base, R);
  } else {
    // all of the thread's loads first (fixed trip count, unrolled): one memory
    // round trip per chunk instead of one per sample
    constexpr int K = CH / NT;
    if constexpr (PR == Pre::Real) {
      const float* __restrict__ x = static_cast<const float*>(a.x) + ch * a.x_stride + base;
      float v[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = threadIdx.x + k * NT;
        v[k] = e < cnt ? x[e] : 0.0f;
      }
#pragma unroll
      for (int k = 0; k < K; ++k) sb[pos(threadIdx.x + k * NT)] = v[k];
    } else {
      const f2* __restrict__ x = static_cast<const f2*>(a.x) + ch * a.x_stride + base;
      f2 v[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = threadIdx.x + k * NT;
        v[k] = e < cnt ? x[e] : f2{0.0f, 0.0f};
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = threadIdx.x + k * NT;
        const f2 z = v[k];
        float o;
        if constexpr (PR == Pre::Ssb) {
          const f2 p = osc_get(a.osc, R, e);
          o = __builtin_fmaf(z.x, p.x, z.y * p.y);  // ssb.rs:37
        } else if constexpr (PR == Pre::AmSqrt) {
          o = __builtin_fmaf(z.x, z.x, z.y * z.y);  // am.rs:204
        } else if constexpr (PR == Pre::AmAbs) {
          o = __builtin_fmaf(a.c.k1, fabsf(z.x), a.c.k2 * fabsf(z.y));  // am.rs:238
        } else {
          o = sqrtf(z.x * z.x + z.y * z.y);  // cw.rs:38
        }
        sb[pos(e)] = o;
      }
    }
  }
}

template <Post PO>
__device__ __forceinline__ float postmap(const ScanArgs& a, float y) {
  if constexpr (PO == Post::Sqrt) return sqrtf(y);  // am.rs:54 process_mapped(.., f32::sqrt)
  else if constexpr (PO == Post::Abs) return fabsf(y);  // process_mapped(.., f32::abs) (iir.rs:170-186)
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

// 4x4-or-smaller f64 matrix product C = A B (one thread).
template <int S>
__device__ void mat_mul_dev(const double* A, const double* B, double* C) {
  for (int r = 0; r < S; ++r)
    for (int c = 0; c < S; ++c) {
      double acc = 0.0;
      for (int k = 0; k < S; ++k) acc = __builtin_fma(A[r * S + k], B[k * S + c], acc);
      C[r * S + c] = acc;
    }
}

// State entering every block of a channel from the block aggregates. Each thread
// owns a run of P = ceil(nblk / NT) consecutive blocks: the run's zero-state
// aggregate (P sequential steps), one workgroup Kogge-Stone over the runs with
// (A^(CH P))^(2^s), then the run walked again writing each block's entering
// state. Runs before the last non-empty one are full, which is all the scan
// needs; later (empty or short) runs write nothing.
template <RecK RK>
__global__ __launch_bounds__(NT) void k_scan_carry(const ScanArgs a, int nblk) {
  constexpr int S = RecSel<RK>::T::S;
  __shared__ double mp[8][S * S];  // (A^(CH P))^(2^s)
  __shared__ double q[2][NT][S];
  const int t = threadIdx.x;
  const int ch = blockIdx.x;
  const int P = (nblk + NT - 1) / NT;
  const double* M1 = a.mats + ScanMatsLayout::kPch * S * S;  // A^CH
  if (t == 0) {  // A^(CH P) by binary powering, then its squarings
    double R[S * S], B[S * S], T2[S * S];
    for (int e = 0; e < S * S; ++e) {
      R[e] = (e / S == e % S) ? 1.0 : 0.0;
      B[e] = M1[e];
    }
    for (int p = P; p > 0; p >>= 1) {
      if (p & 1) {
        mat_mul_dev<S>(R, B, T2);
        for (int e = 0; e < S * S; ++e) R[e] = T2[e];
      }
      if (p > 1) {
        mat_mul_dev<S>(B, B, T2);
        for (int e = 0; e < S * S; ++e) B[e] = T2[e];
      }
    }
    for (int e = 0; e < S * S; ++e) mp[0][e] = R[e];
    for (int sq = 1; sq < 8; ++sq) mat_mul_dev<S>(mp[sq - 1], mp[sq - 1], mp[sq]);
  }
  const int b0 = min(nblk, t * P), b1 = min(nblk, b0 + P);
  const double* __restrict__ ag = a.aggs + static_cast<long long>(ch) * nblk * S;
  double g[S];
#pragma unroll
  for (int i = 0; i < S; ++i) g[i] = 0.0;
#pragma unroll 8
  for (int b = b0; b < b1; ++b) {  // g <- A^CH g + agg_b (unrolled: the loads go out together)
    double v[S];
#pragma unroll
    for (int i = 0; i < S; ++i) v[i] = ag[static_cast<long long>(b) * S + i];
    matvec_acc<S>(M1, g, v);
#pragma unroll
    for (int i = 0; i < S; ++i) g[i] = v[i];
  }
  double carry[S];
#pragma unroll
  for (int i = 0; i < S; ++i) carry[i] = a.carry_in[ch * kScanCarry + i];
  __syncthreads();  // mp ready
  if (t == 0) matvec_acc<S>(mp[0], carry, g);  // fold the incoming state into run 0 (a full run)
  int buf = 0;
  for (int s = 0; s < 8; ++s) {
    const int d = 1 << s;
#pragma unroll
    for (int i = 0; i < S; ++i) q[buf][t][i] = g[i];
    __syncthreads();
    if (t >= d) {
      double o[S];
#pragma unroll
      for (int i = 0; i < S; ++i) o[i] = q[buf][t - d][i];
      matvec_acc<S>(mp[s], o, g);
    }
    buf ^= 1;
  }
#pragma unroll
  for (int i = 0; i < S; ++i) q[buf][t][i] = g[i];
  __syncthreads();
  double st[S];
#pragma unroll
  for (int i = 0; i < S; ++i) st[i] = t == 0 ? carry[i] : q[buf][t - 1][i];
  double* __restrict__ out = a.sin + static_cast<long long>(ch) * nblk * S;
#pragma unroll 8
  for (int b = b0; b < b1; ++b) {  // entering state of each block of the run
    double v[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
      out[static_cast<long long>(b) * S + i] = st[i];
      v[i] = ag[static_cast<long long>(b) * S + i];
    }
    matvec_acc<S>(M1, st, v);
#pragma unroll
    for (int i = 0; i < S; ++i) st[i] = v[i];
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
      OscRun R{};
      if constexpr (PR == Pre::Fm)
        if (a.translate) R = osc_run(a.osc, static_cast<uint64_t>(a.k0 + base), cnt);
      const f2 z = cin<PR>(a, x, a.n - 1, base, R);
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


// ---- single-pass LpDcCascade (SsbProductDemod, AmEnvelopeDemod AbsApprox) ----
// One workgroup per chunk of one channel, the grid chunk-major (blockIdx.x =
// c * nch + ch), so every chunk's predecessor was dispatched earlier. The input
// is read once (the three-kernel scan reads it twice):
//   * LP4: the chunk's 4096 staged samples start kSpWarm samples before its
//     first output, from a zero state (the LP poles decay below 1e-10 of the
//     state within kSpWarm samples: the host checks ||A_lp^kSpWarm||); chunk 0
//     has no warm-up and starts from the carried state. Block-level scan as in
//     k_scan_apply, then the reference's f32 update re-run -> exact LP output x.
//   * DC blocker (y = x - x1 + r y1, pole ~1 - 2.6e-4: it never forgets): a
//     1-dim scan of (r^len, zero-state aggregate) pairs inside the block and a
//     decoupled look-back across chunks (thread 0): each chunk publishes its
//     aggregate, then its inclusive prefix; the state entering chunk c is read
//     from the nearest predecessor that has published a prefix.
// Look-back records (u32 words, agent-scope sc1 stores + flags): [0,2) zero-
// state aggregate, [2,4) r^len, [4,6) inclusive prefix, 6 flag(aggregate),
// 7 flag(prefix); flags hold the launch epoch.
__device__ __forceinline__ void sp_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t sp_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sp_st64(uint32_t* p, double v) {
  const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v));
  sp_st(p, static_cast<uint32_t>(b));
  sp_st(p + 1, static_cast<uint32_t>(b >> 32));
}
__device__ __forceinline__ double sp_ld64(const uint32_t* p) {
  const unsigned long long lo = sp_ld(p), hi = sp_ld(p + 1);
  return __longlong_as_double(static_cast<long long>((hi << 32) | lo));
}
// Bounded wait until flag f1 or f2 holds `epoch`: at most `spin` polls (0: give up at
// once, test-only). false on timeout: the caller flags the handle's error word (the
// record it then reads may be stale; the host reports the call as failed).
__device__ __forceinline__ bool sp_wait2(const uint32_t* f1, const uint32_t* f2, uint32_t epoch, uint32_t spin) {
  for (uint32_t it = 0; it < spin; ++it) {
    if (sp_ld(f1) == epoch || sp_ld(f2) == epoch) return true;
    __builtin_amdgcn_s_sleep(2);
  }
  return false;
}
// (m1, d1) then (m2, d2): y -> m2 (m1 y + d1) + d2
__device__ __forceinline__ void dc_combine(double m1, double d1, double& m2, double& d2) {
  d2 = __builtin_fma(m2, d1, d2);
  m2 = m2 * m1;
}

// Staging of k_lpdc_sp at SC samples per lane, wave-local: wave w stages the chunk's
// elements [64 SC w, 64 SC (w + 1)) (lane l: e = 64 SC w + l + 64 k, coalesced), which
// are exactly the lane runs its own lanes process, so no workgroup barrier separates
// the staging, the LP4 re-run's rewrite and the output staging from their readers (a
// wave's LDS operations execute in order). The SSB mixing phasor of element e is the
// BFO's output k0 + base + e: the reference's from its table, or in the drift model
// (S mtab[64 SC w + l]) mtab[64 k] scaled by the linear magnitude model.
template <int SC>
__device__ __forceinline__ int posS(int e) { return e + static_cast<int>(static_cast<unsigned>(e) / SC); }
// posS(e0 + R k) for e0 >= 0 and SC | R: posS(e0) + k (R + R / SC), so that the row
// offset folds into the LDS instruction's immediate (the division is not redone per row)
template <int SC, int R>
__device__ __forceinline__ int posS_row(int pe0, int k) { return pe0 + k * (R + R / SC); }
__device__ __forceinline__ void wave_order() { asm volatile("" ::: "memory"); }
template <Pre PR, int SC>
__device__ __forceinline__ void stage_sp(const ScanArgs& a, int ch, long long base, int cnt, float* sb) {
  constexpr int WR = 64 * SC;  // elements per wave
  static_assert(kScanCH % WR == 0 && SC * NT <= 2 * kScanCH, "wave ranges inside one phasor table span");
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e0 = w * WR + l;
  if constexpr (PR == Pre::Real || PR == Pre::RealLp || PR == Pre::RealLpSqrt || PR == Pre::RealLpAbs) {  // f32 input
    const float* __restrict__ xr = static_cast<const float*>(a.x) + ch * a.x_stride + base;
    float v[SC];
#pragma unroll
    for (int k = 0; k < SC; ++k) {
      const int e = e0 + 64 * k;
      v[k] = e < cnt ? xr[e] : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < SC; ++k) sb[posS_row<SC, 64>(posS<SC>(e0), k)] = v[k];
    return;
  }
  const f2* __restrict__ x = static_cast<const f2*>(a.x) + ch * a.x_stride + base;
  f2 v[SC];
#pragma unroll
  for (int k = 0; k < SC; ++k) {
    const int e = e0 + 64 * k;
    v[k] = e < cnt ? x[e] : f2{0.0f, 0.0f};
  }
  if constexpr (PR == Pre::Ssb) {
    // the BFO's outputs over the chunk: one tile-uniform branch per form, so only one
    // form's temporaries are live beside v[]
    const OscRun R = osc_run(a.osc, static_cast<uint64_t>(a.k0 + base), cnt);
    const int pe0 = posS<SC>(e0);
    auto put = [&](int k, f2 p) {
      sb[posS_row<SC, 64>(pe0, k)] = __builtin_fmaf(v[k].x, p.x, v[k].y * p.y);  // ssb.rs:37
    };
    if (R.kind == 0) {
#pragma unroll
      for (int k = 0; k < SC; ++k) put(k, osc_tab(a.osc, R, e0 + 64 * k));
    } else if (R.kind == 1) {
      const f2 St = cmul(R.S, a.osc.mtab[e0]);  // the model: (S mtab[e0]) mtab[64 k]
      OscRun Rt = R;
      Rt.S = St;
#pragma unroll
      for (int k = 0; k < SC; ++k) put(k, osc_model(a.osc, Rt, e0 + 64 * k, a.osc.mtab[64 * k]));
    } else {
#pragma unroll
      for (int k = 0; k < SC; ++k) put(k, osc_get(a.osc, R, e0 + 64 * k));
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < SC; ++k) {
    const f2 z = v[k];
    float o;
    if constexpr (PR == Pre::AmSqrt) {
      o = __builtin_fmaf(z.x, z.x, z.y * z.y);  // am.rs:204
    } else {
      o = __builtin_fmaf(a.c.k1, fabsf(z.x), a.c.k2 * fabsf(z.y));  // am.rs:238
    }
    sb[posS_row<SC, 64>(posS<SC>(e0), k)] = o;
  }
}

template <Pre PR, int SC>
__global__ __launch_bounds__(NT, SC > 16 ? kSpMinW : kSpMinW16) void k_lpdc_sp(const ScanArgs a, const double* __restrict__ mlp, int nch,
                                               uint32_t* __restrict__ rec, uint32_t epoch) {
  constexpr int S = 4;
  constexpr int C = SC, CH = SC * NT, PADN = CH + CH / SC + SC;
  // matrices of the lane step A^C: (A^C)^(2^s) are kPwc + s (C = kScanC) or kPwc + 1 + s
  // (C = 2 kScanC: the same powers shifted by one; s = 5 is then kM64); A^(64 C) per wave
  static_assert(SC == kScanC || SC == 2 * kScanC, "lane run");
  constexpr int kPw = ScanMatsLayout::kPwc + (SC == kScanC ? 0 : 1);
  [[maybe_unused]] constexpr int kWv = SC == kScanC ? ScanMatsLayout::kM64 : ScanMatsLayout::kM128;
  __shared__ float sb[PADN];
  __shared__ double tot[4][S];
  __shared__ double dtot[4][2];
  __shared__ float xlast[4];  // each wave's last element (the DC pass's x before the next wave)
  __shared__ double excl_sh;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int ch = static_cast<int>(blockIdx.x % nch);
  const int c = static_cast<int>(blockIdx.x / nch);
  // PR == Real: the DcBlocker alone (no LP4, no warm-up, chunks abut); its state
  // (x1, y1) sits at carry [0, 1] (RecDC) instead of [4, 5] (RecLpDc)
  constexpr bool LP = PR != Pre::Real;
  constexpr int WARM = LP ? kSpWarm : 0, DX = LP ? 4 : 0, DY = DX + 1;
  const int warm = c == 0 ? 0 : WARM;
  const long long o0 = c == 0 ? 0 : CH + static_cast<long long>(c - 1) * (CH - WARM);
  const long long base = o0 - warm;                          // first staged sample
  const int cnt = static_cast<int>(min(static_cast<long long>(CH), a.n - base));  // staged samples
  const int nchunk = a.n <= CH ? 1 : 1 + static_cast<int>((a.n - CH + (CH - WARM) - 1) / (CH - WARM));
  const bool last = c == nchunk - 1;
  const float* __restrict__ ci = a.carry_in + ch * kScanCarry;
  const RecLP4 lp{{a.c.b0, a.c.b1, a.c.b2, a.c.a1, a.c.a2}};
  const float r = a.c.r;
  stage_sp<PR, SC>(a, ch, base, cnt, sb);
  wave_order();  // wave-local staging

  // ---- LP4: zero-state lane aggregates, block scan, exact re-run ----
  // The per-sample loops run unguarded over the lane's C staged samples: the lane's valid
  // samples are i < hi, the staged samples past cnt are zeros, and the recurrences are
  // causal, so what runs past cnt reaches only outputs past cnt (never stored) and the
  // pairs of lanes past cnt. The call's carried state, taken at sample cnt - 1, is
  // re-derived by the lane holding it (last chunk only; `carry_lane`).
  const int hi = min(cnt - t * C, C);
  const bool full_nl = cnt == CH && !last;
  const int il = cnt - 1 - t * C;  // the call's last sample in this lane's run (last chunk)
  const bool carry_lane = last && il >= 0 && il < C;
  float xs[C];
#pragma unroll
  for (int i = 0; i < C; ++i) xs[i] = sb[posS<SC>(t * C + i)];
  float ef[S] = {0, 0, 0, 0};
  if constexpr (LP) {
  float s0[S] = {0, 0, 0, 0};
  {  // the lane run's zero-state end state as the linear map (k_scan_sp)
    const auto E = uniform_table(a.zmap);
#pragma unroll
    for (int i = 0; i < C; ++i)
#pragma unroll
      for (int k = 0; k < S; ++k) s0[k] = __builtin_fmaf(E[i * S + k], xs[i], s0[k]);  // zeros past cnt (staging)
  }
  double q[S];
#pragma unroll
  for (int i = 0; i < S; ++i) q[i] = s0[i];
  double e[S];
  // Truncated scan: the LP4 forgets its state within kSpWarm samples (the host checks
  // ||A^kSpWarm|| < 1e-10, the warm-up's own criterion), i.e. within NL lane runs, so
  // the state entering lane L is sum_{i = 1..NL} A^{C(i-1)} s0[L - i] to that bound:
  // a log2(NL)-step scan over the wave (not 6 steps twice), the previous wave's last
  // inclusive sum Q (lane 63) carried into lanes L < NL as A^{CL} Q, and in chunk 0 the
  // carried state as A^{CL} carry (kLane holds A^{16 m}).
  constexpr int NL = kSpWarm / SC;
  constexpr int STEPS = NL == 8 ? 3 : NL == 16 ? 4 : 5;
  static_assert(NL == (1 << STEPS) && NL * SC / kScanC < 64, "truncated scan geometry");
#pragma unroll 1
  for (int st = 0; st < STEPS; ++st) {
    double o[S];
#pragma unroll
    for (int i = 0; i < S; ++i) o[i] = __shfl_up(q[i], 1 << st, 64);
    if (lane >= (1 << st)) matvec_acc<S>(mlp + (kPw + st) * S * S, o, q);
  }
  if (lane == 63)
#pragma unroll
    for (int i = 0; i < S; ++i) tot[wave][i] = q[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const double o = __shfl_up(q[i], 1, 64);
    e[i] = lane == 0 ? 0.0 : o;
  }
  if (lane < NL && (wave > 0 || c == 0)) {
    double v[S];
#pragma unroll
    for (int i = 0; i < S; ++i) v[i] = wave > 0 ? tot[wave - 1][i] : static_cast<double>(ci[i]);
    matvec_acc<S>(mlp + (ScanMatsLayout::kLane + lane * (SC / kScanC)) * S * S, v, e);
  }
#pragma unroll
  for (int i = 0; i < S; ++i) ef[i] = static_cast<float>(e[i]);
  if (carry_lane) {  // the LP4 state after sample cnt - 1 (the staged inputs are still in sb)
    float e2[S] = {ef[0], ef[1], ef[2], ef[3]};
#pragma unroll 1
    for (int i = 0; i <= il; ++i) (void)lp.step(e2, sb[posS<SC>(t * C + i)]);
    float* co = a.carry_out + ch * kScanCarry;
#pragma unroll
    for (int i = 0; i < S; ++i) co[i] = e2[i];
  }
#pragma unroll
  for (int i = 0; i < C; ++i) {
    xs[i] = lp.step(ef, xs[i]);  // LP output x (f32, reference update)
    if constexpr (PR == Pre::AmSqrt || PR == Pre::RealLpSqrt) xs[i] = sqrtf(xs[i]);  // process_mapped(.., f32::sqrt)
    if constexpr (PR == Pre::RealLpAbs) xs[i] = fabsf(xs[i]);                          // process_mapped(.., f32::abs)
  }
  wave_order();  // (the wave's own inputs: read before they are overwritten, in order)
#pragma unroll
  for (int i = 0; i < C; ++i) sb[posS<SC>(t * C + i)] = xs[i];
  wave_order();
  }  // LP

  // ---- DC blocker: zero-state lane pairs (r^k, y_k), block scan ----
  // x before the lane's first sample: lane 0 of chunk 0 takes the carried x1; lane 0 of a
  // later chunk the sample before the chunk (with the LP4 that sample's position is a
  // warm-up sample, which the DC pass skips). Lane 0 of wave w > 0 needs wave w - 1's last
  // element: it runs its zero-state pass with x_prev = 0 and, after the totals barrier,
  // corrects its pair (y_k shifts by x_prev r^k, so d by x_prev m / r, and every later
  // lane's inclusive pair by x_prev mi / r; the wave's total likewise) — no barrier for it.
  const bool xcross = wave > 0 && lane == 0;
  float xprev0 = t * C == 0 ? ci[DX] : (xcross ? 0.0f : sb[posS<SC>(t * C - 1)]);
  if constexpr (!LP)
    if (t == 0 && c > 0) xprev0 = static_cast<const float*>(a.x)[ch * a.x_stride + base - 1];
  double m = 1.0, d = 0.0;
  // the warm-up is a whole number of lane runs: a lane is inside it or past it
  const bool lane_on = t * C >= warm;
  {
    float y = 0.0f;
    {
      float xp = xprev0;
#pragma unroll
      for (int i = 0; i < C; ++i) {
        y = (xs[i] - xp) + r * y;
        xp = xs[i];
      }
    }
    d = lane_on ? static_cast<double>(y) : 0.0;
    // r^v over the lane's v valid samples by squaring (equal to the running product to
    // f64 rounding, ~1e-15 relative: far below the f32 outputs)
    const int v = lane_on ? max(hi, 0) : 0;
    double p = static_cast<double>(r);
#pragma unroll
    for (int b = 1; b <= C; b <<= 1) {
      if (v & b) m *= p;
      p *= p;
    }
  }
  // inclusive scan of (m, d) over the wave, then over the waves
  double mi = m, di = d;
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int dd = 1 << s;
    const double mo = __shfl_up(mi, dd, 64), do_ = __shfl_up(di, dd, 64);
    if (lane >= dd) dc_combine(mo, do_, mi, di);
  }
  if (lane == 63) {
    dtot[wave][0] = mi;
    dtot[wave][1] = di;
    xlast[wave] = xs[C - 1];
  }
  __syncthreads();
  constexpr int WR = 64 * SC;  // elements per wave
  static_assert(WARM <= WR, "xcorr: lane 0 of a wave w > 0 must sit past the LP4 warm-up");
  const double rd = static_cast<double>(r);
  // the x_prev correction of wave w's pairs (lane 0 of a wave holds a valid sample iff
  // the wave does: its first element is past the warm-up)
  auto xcorr = [&](int w) -> double { return (w > 0 && w * WR < cnt) ? static_cast<double>(xlast[w - 1]) : 0.0; };
  // r^(v - 1) from a pair's multiplier r^v over v >= 1 valid samples. r = 0 is a real
  // design (dc.rs:17 / iir.rs:122 clamp a cut >= fs / 2 pi to 0): then only y_0 sees x_prev.
  auto over_r = [&](double mprod, int v) -> double { return rd != 0.0 ? mprod / rd : (v == 1 ? 1.0 : 0.0); };
  {
    const double xw = xcorr(wave);
    if (xw != 0.0) di -= xw * over_r(mi, min((lane + 1) * C, cnt - wave * WR));
    if (xcross) xprev0 = static_cast<float>(xw);
  }
  auto wave_pair_d = [&](int w) -> double {
    const double xw = xcorr(w);
    return xw != 0.0 ? dtot[w][1] - xw * over_r(dtot[w][0], min(WR, cnt - w * WR)) : dtot[w][1];
  };
  double wm = 1.0, wd = 0.0;  // pairs of the waves before this one
  for (int w = 0; w < wave; ++w) {
    double m2 = dtot[w][0], d2 = wave_pair_d(w);
    dc_combine(wm, wd, m2, d2);
    wm = m2;
    wd = d2;
  }
  if (wave == 0) {  // chunk aggregate, look-back (one wave, 64 predecessors per step), prefix
    double bm = 1.0, bd = 0.0;
    for (int w = 0; w < 4; ++w) {
      double m2 = dtot[w][0], d2 = wave_pair_d(w);
      dc_combine(bm, bd, m2, d2);
      bm = m2;
      bd = d2;
    }
    uint32_t* my = rec + (static_cast<long long>(ch) * nchunk + c) * 8;
    if (!last) {
      if (lane == 0) {
        sp_st64(my, bd);
        sp_st64(my + 2, bm);
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the record is visible before its flag
      if (lane == 0) sp_st(my + 6, epoch);
    }
    // lane i looks at chunk k = base - i; the nearest chunk with a prefix (or
    // the carried state before chunk 0) closes the walk:
    //   excl = sum_{i <= first} (prod_{j < i} r^len_j) v_i
    double excl = 0.0, mult = 1.0;
    // The DC blocker forgets too, only slowly: r^len ~ 0.12 per 7936-sample chunk at
    // 2 Hz / 48 kHz. Past K chunks, with r^(K len) < 1e-20, what entered them cannot reach
    // this chunk's f32 outputs: the walk treats chunk c-1-K as a zero state (no wait on it
    // or beyond), and ends at latest once the walked product of r^len is below 1e-20.
    const float lr = static_cast<float>(CH - warm) * __logf(r);
    const int K = !(r > 0.0f) ? 1 : (lr < 0.0f ? static_cast<int>(min(64.0f, ceilf(-46.06f / lr))) : 64);
    for (int base = c - 1;; base -= 64) {
      const int k = base - lane;
      double v = 0.0, mk = 1.0;
      bool closes = true;
      if (base == c - 1 && lane >= K) {
        // past the horizon: a zero state closes the walk (v = 0)
      } else if (k >= 0) {
        const uint32_t* pr = rec + (static_cast<long long>(ch) * nchunk + k) * 8;
        if (!sp_wait2(pr + 6, pr + 7, epoch, a.spin)) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        closes = sp_ld(pr + 7) == epoch;
        v = closes ? sp_ld64(pr + 4) : sp_ld64(pr);
        mk = closes ? 1.0 : sp_ld64(pr + 2);
      } else {
        v = static_cast<double>(ci[DY]);  // the carried y1
      }
      const unsigned long long bal = __ballot(closes);
      const int first = bal ? __builtin_ctzll(bal) : 64;
      // exclusive product of the multipliers over lanes (multiplicative scan)
      double pm = mk;
#pragma unroll
      for (int s2 = 0; s2 < 6; ++s2) {
        const double o = __shfl_up(pm, 1 << s2, 64);
        if (lane >= (1 << s2)) pm *= o;
      }
      double ep = __shfl_up(pm, 1, 64);
      if (lane == 0) ep = 1.0;
      double term = lane <= first ? ep * v : 0.0;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) term += __shfl_xor(term, off, 64);
      excl = __builtin_fma(mult, term, excl);
      if (first < 64) break;
      mult *= __shfl(pm, 63, 64);
      if (!(fabs(mult) >= 1e-20)) break;
    }
    if (!last && lane == 0) {
      sp_st64(my + 4, __builtin_fma(bm, excl, bd));
      __builtin_amdgcn_s_waitcnt(0x0F70);
      sp_st(my + 7, epoch);
    }
    if (lane == 0) excl_sh = excl;
  }
  __syncthreads();
  // the state entering this lane: exclusive pair within the block applied to excl
  double em = __shfl_up(mi, 1, 64), ed = __shfl_up(di, 1, 64);
  if (lane == 0) {
    em = 1.0;
    ed = 0.0;
  }
  dc_combine(wm, wd, em, ed);  // waves before, then lanes before
  float y = static_cast<float>(__builtin_fma(em, excl_sh, ed));
  {  // (warm-up lanes' outputs are not stored)
    float xp = xprev0;
#pragma unroll
    for (int i = 0; i < C; ++i) {
      y = (xs[i] - xp) + r * y;  // dsp/iir.rs:161 (y1 - dc_x1) + r * dc_y1
      xp = xs[i];
      xs[i] = y;
    }
  }
  // carried state of the next call: x1 = the LP output at sample cnt - 1 (still in sb),
  // y1 = the output there
  const float xl = carry_lane ? sb[posS<SC>(cnt - 1)] : 0.0f;
  wave_order();  // output staging, wave-local (every cross-wave read of sb was before the last barrier)
#pragma unroll
  for (int i = 0; i < C; ++i) sb[posS<SC>(t * C + i)] = xs[i];
  wave_order();
  if (carry_lane) {
    float* co = a.carry_out + ch * kScanCarry;
    co[DX] = xl;
    co[DY] = sb[posS<SC>(cnt - 1)];
    co[6] = ci[6];
    co[7] = ci[7];
  }
  float* yo = static_cast<float*>(a.y) + ch * a.y_stride + o0;
  const int e0 = wave * (64 * SC) + lane;
  if (full_nl) {
    const int kmin = (warm - wave * (64 * SC)) >> 6;  // wave-uniform: the warm-up is whole rows of 64
#pragma unroll
    for (int k = 0; k < SC; ++k)
      if (k >= kmin) yo[e0 + 64 * k - warm] = sb[posS_row<SC, 64>(posS<SC>(e0), k)];
  } else {
#pragma unroll
    for (int k = 0; k < SC; ++k) {
      const int e2 = e0 + 64 * k;
      if (e2 >= warm && e2 < cnt) yo[e2 - warm] = sb[posS_row<SC, 64>(posS<SC>(e0), k)];
    }
  }
}

// ---- single-pass scan for recurrences that forget (k_scan_sp) ---------------------
// LpCascade and the demodulators built on it (FM, PM, AM PowerSqrt) and the CW
// one-pole, when the chunk transition A^CH is negligible (the host checks
// ||A^kSpCH|| < 1e-10: whatever state enters chunk c-1 is gone by its end), so the
// state entering chunk c is chunk c-1's zero-state end state. Every chunk publishes
// that aggregate as soon as its zero-state pass and block scan are done, then reads
// its predecessor's (chunk-major grid: the predecessor was dispatched earlier and
// publishes before it waits, so no chain of waits forms). Against the three-kernel
// scan this drops the carry pass and the second read of the input. kSpC samples per
// lane as k_lpdc_sp. Records: 16 u32 per (channel, chunk), [0, 2S) the aggregate
// (f64), 15 the flag (launch epoch).
// TRS > 0: the stage also forgets within H = 2^TRS lane runs (H C samples; the host
// picks the smallest H in {256, 512, 1024} samples with ||A^H|| < 1e-10): the lane scan
// truncated to TRS steps, as in k_lpdc_sp. TRS = 0: the full scan and re-scan.
template <RecK RK, Pre PR, Post PO, int TRS>
__global__ __launch_bounds__(NT, kScanSpMinW) void k_scan_sp(const ScanArgs a, int nch, uint32_t* __restrict__ rec,
                                                   uint32_t epoch) {
  using R = typename RecSel<RK>::T;
  constexpr int S = R::S;
  constexpr int SC = kSpC, C = SC, CH = SC * NT, PADN = CH + CH / SC + SC;
  constexpr int kPw = ScanMatsLayout::kPwc + 1;    // (A^C)^(2^s), C = 2 kScanC
  constexpr int kWv = ScanMatsLayout::kM128;       // A^(64 C)
  __shared__ float sb[PADN];
  __shared__ double tot[4][S];
  __shared__ double cin_sh[S];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int ch = static_cast<int>(blockIdx.x % nch);
  const int c = static_cast<int>(blockIdx.x / nch);
  const long long base = static_cast<long long>(c) * CH;
  const int cnt = static_cast<int>(min(static_cast<long long>(CH), a.n - base));
  const int nchunk = static_cast<int>((a.n + CH - 1) / CH);
  const bool last = c == nchunk - 1;
  const float* __restrict__ ci = a.carry_in + ch * kScanCarry;
  const R rr = RecSel<RK>::make(a.c);
  OscRun Ro{};  // the translator's outputs of the chunk
  if constexpr (PR == Pre::Fm)
    if (a.translate) Ro = osc_run(a.osc, static_cast<uint64_t>(a.k0 + base), cnt);
  // Batches of 8 samples per thread: every load of a batch issued before any is used
  // (unconditional, index clamped into [0, n)), then the pre-map. (A guarded load per
  // sample compiles to a branch around each, which waits for its load before the LDS
  // store: one memory latency per sample.) FM / PM also load x[i - 1] (an L1/L2 hit).
  constexpr int BT = PR == Pre::Real ? kSpBatchReal : PR == Pre::Pm ? 8 : kSpBatch;  // loads per thread at once
  static_assert(SC % BT == 0 && BT <= 64 && CH <= kOscSpan, "staging batches; one oscillator cursor per chunk");
  // FM: the previous sample from the neighbour lane (below); PM: its own load of x[i - 1]
  // (an L1/L2 hit; the neighbour form measured 6 % slower there: more spills)
  constexpr bool kPair = PR == Pre::Fm, kPrev = PR == Pre::Pm;
  const long long nl = a.n - 1;
  // a full chunk that is not the call's last: no index clamps, no store guards (below)
  const bool fast = cnt == CH && !last;
  auto stage = [&](auto guarded) {
  constexpr bool G = decltype(guarded)::value;
#pragma unroll 1
  for (int k0 = 0; k0 < SC; k0 += BT) {
    f2 z[BT], zp[BT], zq = f2{0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < BT; ++j) {
      const long long i = base + t + (k0 + j) * NT;
      if constexpr (PR == Pre::Real) {
        z[j] = f2{static_cast<const float*>(a.x)[ch * a.x_stride + (G ? min(i, nl) : i)], 0.0f};
      } else {
        const f2* __restrict__ xc = static_cast<const f2*>(a.x) + ch * a.x_stride;
        z[j] = xc[G ? min(i, nl) : i];
        zp[j] = kPrev ? xc[G || c == 0 ? max(min(i - 1, nl), 0LL) : i - 1] : z[j];
      }
    }
    if constexpr (kPair) {
      // FM: the previous sample of lane L is lane L - 1's (a DPP shift of the mapped
      // sample: no second load, no second translation); lane 0 of the wave needs the sample before the wave's run of
      // row k0 + j: lane j of the wave loads and maps it for all eight j in one load.
      const long long iq = base + (t & ~63) + (k0 + (lane % BT)) * NT - 1;
      zq = cin_v<PR>(a, (static_cast<const f2*>(a.x) + ch * a.x_stride)[max(min(iq, nl), 0LL)], iq, base, Ro);
    }
#pragma unroll
    for (int j = 0; j < BT; ++j) {
      const int e = t + (k0 + j) * NT;
      float o;
      if constexpr (kPair) {
        const f2 zc = cin_v<PR>(a, z[j], base + e, base, Ro);
        f2 p = f2{wave_up<1>(zc.x), wave_up<1>(zc.y)};
        if (lane == 0) {
          p = f2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(zq.x), j)),
                 __int_as_float(__builtin_amdgcn_readlane(__float_as_int(zq.y), j))};
          if (base + e == 0) p = f2{ci[6], ci[7]};  // the carried previous sample
        }
        o = fm_disc(zc, p, a.c.k);
      } else {
        o = premap_v<PR>(a, ch, base + e, base, Ro, z[j], zp[j]);
      }
      sb[posS_row<SC, NT>(posS<SC>(t), k0 + j)] = !G || e < cnt ? o : 0.0f;  // e = t + (k0 + j) NT
    }
  }
  };
  if (fast) stage(std::false_type{});
  else stage(std::true_type{});
  __syncthreads();

  // The per-sample loops run unguarded (as k_lpdc_sp): samples past cnt are staged as
  // zeros, and what the causal recurrence computes past cnt reaches only outputs past cnt
  // (never stored); the lane holding sample cnt - 1 re-derives the carried state.
  const int il = cnt - 1 - t * C;
  const bool carry_lane = last && il >= 0 && il < C;
  float xs[C];
#pragma unroll
  for (int i = 0; i < C; ++i) xs[i] = sb[posS<SC>(t * C + i)];
  float s0[S];
#pragma unroll
  for (int i = 0; i < S; ++i) s0[i] = 0.0f;
  {
    // the lane run's zero-state end state as the linear map sum_i A^(C-1-i) B x_i
    // (independent FMAs instead of the recurrence's dependent chain; samples past the
    // chunk enter as zeros: only the last partial lane differs, whose state reaches no
    // valid output)
    const auto E = uniform_table(a.zmap);
#pragma unroll
    for (int i = 0; i < C; ++i)
#pragma unroll
      for (int k = 0; k < S; ++k) s0[k] = __builtin_fmaf(E[i * S + k], xs[i], s0[k]);
  }
  double q[S];
#pragma unroll
  for (int i = 0; i < S; ++i) q[i] = s0[i];
  constexpr bool TR = TRS > 0;
  constexpr int NL = 1 << TRS;
  static_assert(TRS <= 5 && NL * (SC / kScanC) <= 64, "truncation horizon within the kLane table");
  if constexpr (TR) {
#pragma unroll 1
    for (int st = 0; st < TRS; ++st) {
      double o[S];
#pragma unroll
      for (int i = 0; i < S; ++i) o[i] = __shfl_up(q[i], 1 << st, 64);
      if (lane >= (1 << st)) matvec_acc<S>(a.mats + (kPw + st) * S * S, o, q);
    }
  } else {
    wave_scan_inclusive<S>(q, a.mats + kPw * S * S, lane);
  }
  if (lane == 63)
#pragma unroll
    for (int i = 0; i < S; ++i) tot[wave][i] = q[i];
  __syncthreads();
  if (t == 0) {
    double agg[S];
#pragma unroll
    for (int i = 0; i < S; ++i) agg[i] = 0.0;
    // truncated: the chunk's last lane already holds its zero-state end state
    for (int w = TR ? 3 : 0; w < 4; ++w) {
      double v[S];
#pragma unroll
      for (int i = 0; i < S; ++i) v[i] = tot[w][i];
      matvec_acc<S>(a.mats + kWv * S * S, agg, v);
#pragma unroll
      for (int i = 0; i < S; ++i) agg[i] = v[i];
    }
    if (!last) {
      uint32_t* my = rec + (static_cast<long long>(ch) * nchunk + c) * 16;
#pragma unroll
      for (int i = 0; i < S; ++i) sp_st64(my + 2 * i, agg[i]);
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the aggregate is visible before its flag
      sp_st(my + 15, epoch);
    }
    if (c == 0) {
#pragma unroll
      for (int i = 0; i < S; ++i) cin_sh[i] = static_cast<double>(ci[i]);
    } else {
      const uint32_t* pr = rec + (static_cast<long long>(ch) * nchunk + c - 1) * 16;
      if (!sp_wait2(pr + 15, pr + 15, epoch, a.spin)) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
      for (int i = 0; i < S; ++i) cin_sh[i] = sp_ld64(pr + 2 * i);
    }
  }
  __syncthreads();
  float ef[S];
  if constexpr (TR) {
    double e[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
      const double o = __shfl_up(q[i], 1, 64);
      e[i] = lane == 0 ? 0.0 : o;
    }
    if (lane < NL) {  // the previous wave's sum, or the state entering the chunk, as A^{C lane} v
      double v[S];
#pragma unroll
      for (int i = 0; i < S; ++i) v[i] = wave > 0 ? tot[wave - 1][i] : cin_sh[i];
      matvec_acc<S>(a.mats + (ScanMatsLayout::kLane + lane * (SC / kScanC)) * S * S, v, e);
    }
#pragma unroll
    for (int i = 0; i < S; ++i) ef[i] = static_cast<float>(e[i]);
  } else {
  double cw[S];
#pragma unroll
  for (int i = 0; i < S; ++i) cw[i] = cin_sh[i];
  for (int w = 0; w < wave; ++w) {
    double v[S];
#pragma unroll
    for (int i = 0; i < S; ++i) v[i] = tot[w][i];
    matvec_acc<S>(a.mats + kWv * S * S, cw, v);
#pragma unroll
    for (int i = 0; i < S; ++i) cw[i] = v[i];
  }
  // the wave's entering state folded into lane 0 and the wave re-scanned (k_lpdc_sp)
#pragma unroll
  for (int i = 0; i < S; ++i) q[i] = s0[i];
  if (lane == 0) matvec_acc<S>(a.mats + kPw * S * S, cw, q);
  wave_scan_inclusive<S>(q, a.mats + kPw * S * S, lane);
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const double o = __shfl_up(q[i], 1, 64);
    ef[i] = static_cast<float>(lane == 0 ? cw[i] : o);
  }
  }  // TR
  if (carry_lane) {  // carried state of the next call: the state after sample cnt - 1
    float e2[S];
#pragma unroll
    for (int i = 0; i < S; ++i) e2[i] = ef[i];
#pragma unroll 1
    for (int i = 0; i <= il; ++i) (void)rr.step(e2, sb[posS<SC>(t * C + i)]);
    float* co = a.carry_out + ch * kScanCarry;
#pragma unroll
    for (int i = 0; i < S; ++i) co[i] = e2[i];
    for (int i = S; i < 6; ++i) co[i] = 0.0f;
    if constexpr (PR == Pre::Fm || PR == Pre::Pm) {
      const f2* x = static_cast<const f2*>(a.x) + ch * a.x_stride;
      const f2 z = cin<PR>(a, x, a.n - 1, base, Ro);
      co[6] = z.x;
      co[7] = z.y;
    } else {
      co[6] = ci[6];
      co[7] = ci[7];
    }
  }
#pragma unroll
  for (int i = 0; i < C; ++i) xs[i] = postmap<PO>(a, rr.step(ef, xs[i]));  // the reference's f32 update
  __syncthreads();
#pragma unroll
  for (int i = 0; i < C; ++i) sb[posS<SC>(t * C + i)] = xs[i];
  __syncthreads();
  float* y = static_cast<float*>(a.y) + ch * a.y_stride + base;
  if (fast) {
#pragma unroll
    for (int k = 0; k < SC; ++k) y[t + k * NT] = sb[posS_row<SC, NT>(posS<SC>(t), k)];
  } else {
    for (int e2 = t; e2 < cnt; e2 += NT) y[e2] = sb[posS<SC>(e2)];
  }
}

// SsbPhasingMod in one pass (modulate/ssb.rs:43-114): per chunk, the audio-NCO
// products of both branches staged in LDS, both LpCascades as LP4 block scans
// (warm-up of kSpWarm samples from a zero state after the first chunk, as in
// k_lpdc_sp: the host checks ||A^kSpWarm||), and (I, side Q) x RF NCO stored.
// carry: [I state 4][Q state 4] floats.
__global__ __launch_bounds__(NT, 3) void k_ssb_mod_sp(const float* __restrict__ x, f2* __restrict__ y, long long n,
                                                   uint64_t k0, const OscDev aud, const OscDev rf, float side,
                                                   ScanCoef cf, const double* __restrict__ mlp,
                                                   const float* __restrict__ zmap,
                                                   const float* __restrict__ carry_in, float* __restrict__ carry_out) {
  constexpr int S = 4;
  __shared__ float sb[2][PADN];
  __shared__ double tot[2][4][S];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c = static_cast<int>(blockIdx.x);
  const int warm = c == 0 ? 0 : kSpWarm;
  const long long o0 = c == 0 ? 0 : CH + static_cast<long long>(c - 1) * (CH - kSpWarm);
  const long long base = o0 - warm;
  const int cnt = static_cast<int>(min(static_cast<long long>(CH), n - base));
  const bool last = o0 + (cnt - warm) >= n;
  const RecLP4 lp{{cf.b0, cf.b1, cf.b2, cf.a1, cf.a2}};
  // Oscillator outputs k0 + base + e of element e = t + k NT (the coalesced order of the
  // staging and of the stores): the audio and RF Rotators' cursors over the chunk.
  const OscRun Ra = osc_run(aud, k0 + static_cast<uint64_t>(base), cnt);
  const OscRun Rr = osc_run(rf, k0 + static_cast<uint64_t>(base), cnt);
  // `fast` (block-uniform: a full chunk that is not the call's last): unguarded copies of
  // the per-sample loops (as k_lpdc_sp)
  const bool fast = cnt == CH && !last;
  auto stage = [&](auto guarded) {  // x p.re, x p.im (ssb.rs:53-54), coalesced loads first
    constexpr bool G = decltype(guarded)::value;
    float v[C];
    f2 pa[C];  // the audio phasor reads (unconditional: the table is padded past a run)
#pragma unroll
    for (int k = 0; k < C; ++k) {
      v[k] = x[G ? min(base + t + k * NT, n - 1) : base + t + k * NT];
      pa[k] = osc_ld(aud, Ra, t + k * NT);
    }
#pragma unroll
    for (int k = 0; k < C; ++k) {
      const int e = t + k * NT;
      const float xv = !G || e < cnt ? v[k] : 0.0f;  // zeros past cnt (the zero-state map below)
      const f2 p = !G || e < cnt ? osc_fin(aud, Ra, e, pa[k]) : f2{1.0f, 0.0f};
      sb[0][pos(e)] = xv * p.x;
      sb[1][pos(e)] = xv * p.y;
    }
  };
  if (fast) stage(std::false_type{});
  else stage(std::true_type{});
  __syncthreads();
  float xs[2][C];
  float s0[2][S];
  double qt[2][S];  // truncated scan (k_lpdc_sp): NL = kSpWarm / C lane runs span the horizon
  constexpr int NL = kSpWarm / C, STEPS = NL == 16 ? 4 : NL == 8 ? 3 : 5;
  static_assert(NL == (1 << STEPS) && NL * C / kScanC < 64, "truncated scan geometry");
#pragma unroll
  for (int b = 0; b < 2; ++b) {
#pragma unroll
    for (int i = 0; i < C; ++i) xs[b][i] = sb[b][pos(t * C + i)];
#pragma unroll
    for (int k = 0; k < S; ++k) s0[b][k] = 0.0f;
#pragma unroll
    for (int i = 0; i < C; ++i)  // the lane run's zero-state end state as the linear map (k_scan_sp)
#pragma unroll
      for (int k = 0; k < S; ++k) s0[b][k] = __builtin_fmaf(zmap[i * S + k], xs[b][i], s0[b][k]);  // staged zeros past cnt
    double q[S];
#pragma unroll
    for (int k = 0; k < S; ++k) q[k] = s0[b][k];
#pragma unroll 1
    for (int st = 0; st < STEPS; ++st) {
      double o[S];
#pragma unroll
      for (int k = 0; k < S; ++k) o[k] = __shfl_up(q[k], 1 << st, 64);
      if (lane >= (1 << st)) matvec_acc<S>(mlp + (ScanMatsLayout::kPwc + st) * S * S, o, q);
    }
#pragma unroll
    for (int k = 0; k < S; ++k) qt[b][k] = q[k];
    if (lane == 63)
#pragma unroll
      for (int k = 0; k < S; ++k) tot[b][wave][k] = q[k];
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    double e[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const double o = __shfl_up(qt[b][k], 1, 64);
      e[k] = lane == 0 ? 0.0 : o;
    }
    if (lane < NL && (wave > 0 || c == 0)) {
      double v[S];
#pragma unroll
      for (int k = 0; k < S; ++k) v[k] = wave > 0 ? tot[b][wave - 1][k] : static_cast<double>(carry_in[4 * b + k]);
      matvec_acc<S>(mlp + (ScanMatsLayout::kLane + lane * (C / kScanC)) * S * S, v, e);
    }
    float ef[S];
#pragma unroll
    for (int k = 0; k < S; ++k) ef[k] = static_cast<float>(e[k]);
    auto rerun = [&](auto guarded) {
#pragma unroll
      for (int i = 0; i < C; ++i)
        if (!decltype(guarded)::value || t * C + i < cnt) xs[b][i] = lp.step(ef, xs[b][i]);  // ssb.rs:53-54 LpCascade outputs
    };
    if (fast) rerun(std::false_type{});
    else rerun(std::true_type{});
    if (last && t * C <= cnt - 1 && cnt - 1 < t * C + C)  // the next call's state
#pragma unroll
      for (int k = 0; k < S; ++k) carry_out[4 * b + k] = ef[k];
  }
  // (I, side Q) staged in LDS (sb is free: every thread read its runs before the totals
  // barrier; 17 f2 per thread: conflict-free b64 stores), then stored coalesced
  // (each thread owning 16 consecutive samples would store 64 lanes x 8 B at a 128-B
  // stride per instruction)
  f2* zs = reinterpret_cast<f2*>(&sb[0][0]);
  static_assert(2 * PADN >= 2 * (CH + CH / 16), "output staging fits");
#pragma unroll
  for (int i = 0; i < C; ++i) zs[17 * t + i] = f2{xs[0][i], side * xs[1][i]};
  __syncthreads();
  f2 pr[C];  // the RF phasor reads, all issued before the first store
#pragma unroll
  for (int k = 0; k < C; ++k) pr[k] = osc_ld(rf, Rr, t + k * NT);
  static_assert(kSpWarm % NT == 0, "the warm-up is whole rows of the store order");
  if (fast) {
#pragma unroll
    for (int k = 0; k < C; ++k) {  // ssb.rs:55-60
      const int e = t + k * NT;
      if (k * NT >= warm) y[base + e] = cmul_rot(zs[e + (e >> 4)], osc_fin(rf, Rr, e, pr[k]));
    }
  } else {
#pragma unroll
    for (int k = 0; k < C; ++k) {  // ssb.rs:55-60
      const int e = t + k * NT;
      if (e >= warm && e < cnt) y[base + e] = cmul_rot(zs[e + (e >> 4)], osc_fin(rf, Rr, e, pr[k]));
    }
  }
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
    case RecK::BQ: return 2;
    default: return 1;
  }
}

void launch_ssb_mod_sp(const float* x, f2* y, long long n, uint64_t k0, const OscDev& aud, const OscDev& rf,
                       float side, const ScanCoef& c, const double* mats_lp, const float* zmap_lp,
                       const float* carry_in, float* carry_out, hipStream_t s) {
  if (n <= 0) return;
  const long long grid = lpdc_sp_chunks(n);
  if (grid > (1LL << 31) - 1) throw HipError("single-pass SSB modulator grid too large");
  k_ssb_mod_sp<<<static_cast<int>(grid), NT, 0, s>>>(x, y, n, k0, aud, rf, side, c, mats_lp, zmap_lp, carry_in,
                                                       carry_out);
  ORION_LAUNCH_CHECK();
}

long long lpdc_sp_chunks(long long n) {
  return n <= CH ? 1 : 1 + (n - CH + (CH - kSpWarm) - 1) / (CH - kSpWarm);
}

long long lpdc_sp_demod_chunks(long long n, int sc, int warm) {
  const long long ch = static_cast<long long>(sc) * NT;
  return n <= ch ? 1 : 1 + (n - ch + (ch - warm) - 1) / (ch - warm);
}

void launch_lpdc_sp(Pre pre, const ScanArgs& a, const double* mats_lp, int nch, uint32_t* rec, uint32_t epoch,
                    hipStream_t s) {
  if (a.n <= 0 || nch <= 0) return;
  const long long grid = lpdc_sp_demod_chunks(a.n, kLpdcSC, pre == Pre::Real ? 0 : kSpWarm) * nch;
  if (grid > (1LL << 31) - 1) throw HipError("single-pass scan grid too large");
  const int g = static_cast<int>(grid);
  if (pre == Pre::Ssb) {
    k_lpdc_sp<Pre::Ssb, kLpdcSC><<<g, NT, 0, s>>>(a, mats_lp, nch, rec, epoch);
  } else if (pre == Pre::AmAbs) {
    k_lpdc_sp<Pre::AmAbs, kLpdcSC><<<g, NT, 0, s>>>(a, mats_lp, nch, rec, epoch);
  } else if (pre == Pre::Real) {
    k_lpdc_sp<Pre::Real, kLpdcSC><<<g, NT, 0, s>>>(a, mats_lp, nch, rec, epoch);
  } else if (pre == Pre::AmSqrt) {
    k_lpdc_sp<Pre::AmSqrt, kLpdcSC><<<g, NT, 0, s>>>(a, mats_lp, nch, rec, epoch);
  } else if (pre == Pre::RealLp) {
    k_lpdc_sp<Pre::RealLp, kLpdcSC><<<g, NT, 0, s>>>(a, mats_lp, nch, rec, epoch);
  } else if (pre == Pre::RealLpSqrt) {
    k_lpdc_sp<Pre::RealLpSqrt, kLpdcSC><<<g, NT, 0, s>>>(a, mats_lp, nch, rec, epoch);
  } else if (pre == Pre::RealLpAbs) {
    k_lpdc_sp<Pre::RealLpAbs, kLpdcSC><<<g, NT, 0, s>>>(a, mats_lp, nch, rec, epoch);
  } else {
    throw std::invalid_argument("single-pass LpDc scan: unsupported front end");
  }
  ORION_LAUNCH_CHECK();
}

long long scan_sp_chunks(long long n) { return (n + kSpCH - 1) / kSpCH; }

bool scan_sp_supported(RecK rec, Pre pre, Post post) {
  return (rec == RecK::LP4 && post == Post::Id && (pre == Pre::Real || pre == Pre::Fm || pre == Pre::Pm)) ||
         (rec == RecK::BQ && pre == Pre::Real && post == Post::Id) ||
         (rec == RecK::LP4 && pre == Pre::AmSqrt && post == Post::Sqrt) ||
         (rec == RecK::ONEPOLE && pre == Pre::Cw && post == Post::Gain);
}

void launch_scan_sp(RecK rec, Pre pre, Post post, const ScanArgs& a, int nch, uint32_t* recs, uint32_t epoch,
                    int trs, hipStream_t s) {
  if (a.n <= 0 || nch <= 0) return;
  const long long grid = scan_sp_chunks(a.n) * nch;
  if (grid > (1LL << 31) - 1) throw HipError("single-pass scan grid too large");
  const int g = static_cast<int>(grid);
#define ORION_SP(RK, PR, PO)                                                                         \
  if (rec == RecK::RK && pre == Pre::PR && post == Post::PO) {                                       \
    if (trs == 3) k_scan_sp<RecK::RK, Pre::PR, Post::PO, 3><<<g, NT, 0, s>>>(a, nch, recs, epoch);   \
    else if (trs == 4) k_scan_sp<RecK::RK, Pre::PR, Post::PO, 4><<<g, NT, 0, s>>>(a, nch, recs, epoch); \
    else if (trs == 5) k_scan_sp<RecK::RK, Pre::PR, Post::PO, 5><<<g, NT, 0, s>>>(a, nch, recs, epoch); \
    else k_scan_sp<RecK::RK, Pre::PR, Post::PO, 0><<<g, NT, 0, s>>>(a, nch, recs, epoch);            \
    ORION_LAUNCH_CHECK();                                                                            \
    return;                                                                                          \
  }
  ORION_SP(LP4, Real, Id)
  ORION_SP(BQ, Real, Id)
  ORION_SP(LP4, Fm, Id)
  ORION_SP(LP4, Pm, Id)
  ORION_SP(LP4, AmSqrt, Sqrt)
  ORION_SP(ONEPOLE, Cw, Gain)
#undef ORION_SP
  throw std::invalid_argument("single-pass scan: unsupported combination");
}

void launch_scan(RecK rec, Pre pre, Post post, const ScanArgs& a, int nch, hipStream_t s) {
  if (a.n <= 0 || nch <= 0) return;
#define ORION_SCAN(RK, PR, PO) \
  if (rec == RecK::RK && pre == Pre::PR && post == Post::PO) return run3<RecK::RK, Pre::PR, Post::PO>(a, nch, s);
  ORION_SCAN(LP4, Real, Id)
  ORION_SCAN(LP4, Real, Sqrt)
  ORION_SCAN(LP4, Real, Abs)
  ORION_SCAN(BQ, Real, Id)
  ORION_SCAN(LPDC, Real, Id)
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
