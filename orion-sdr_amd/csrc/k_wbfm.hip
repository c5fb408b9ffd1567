// k_wbfm.hip — the WBFM demodulation chain on gfx950 (the north-star path).
//
// Reference composition (docs/demodulate.md:128-133, SURVEY §3 stack 2):
//   Rotator(-f_off).rotate_block (dsp/rotator.rs:74-85)
//   -> FirDecimator(fs, 8, ...)  (dsp/decim.rs:44-76; kept outputs only here)
//   -> FmQuadratureDemod         (demodulate/fm.rs:45-77: discriminator + LpCascade)
//   -> FirLowpass                (dsp/fir.rs:47-66, the audio filter).
//
// Building blocks (one 64-lane wave each, no workgroup barriers):
//   front tile (fu_tile8) — 1024 cf32 inputs -> 128 decimated outputs: the tile's
//     inputs were prefetched one tile ahead (16-B nontemporal loads into
//     registers), are NCO-mixed with per-lane phasors and scattered into an
//     8-row polyphase LDS image (17-column halo carried from the previous tile),
//     the 127-tap polyphase FIR runs at the kept outputs (eight per lane over the
//     four ds_read_b128 lane groups, packed FMA, taps from LDS), the tile's common
//     phasor multiplies them, and the discriminator (atan2_approx op for op, the
//     ratio from v_rcp_f32) writes 128 phi.
//   sub-range back — LpCascade over 1024 phi (iir16: a zero-state packed pass,
//     one f64 Kogge-Stone over the wave, then the reference's f32 TDF-II
//     recurrence into f16 hi / lo planes scaled per sub-range); audio FIR = 125
//     taps as Toeplitz products on v_mfma_f32_16x16x32_f16 (three products per
//     K-step, f32 accumulation), A operands from LDS (sg::back).
// Kernels:
//   k_wbfm_seg (default) — one round of waves, each walking a segment of 1024-
//     output sub-ranges (see the comment at the kernel).
//   k_wbfm_front2 + k_wbfm_back — the two-kernel path (phi through HBM, a
//     510-sample IIR warm-up per 2048 outputs): any IIR design, used when the
//     LpCascade decays too slowly for the segment hand-offs (ORION_WBFM_SPLIT).
// The first tile / sub-range of each channel starts from the exact state carried
// from the previous call (last decimated sample, 128 raw inputs, IIR state, last
// 128 IIR outputs), so k calls equal one call on the concatenation.
#include <algorithm>
#include <cstdlib>

#include "iir.hpp"
#include "kernels.hpp"
#include "poly.hpp"

namespace orion {
namespace {

// Ordering of a wave's own LDS hand-offs (a write, then reads of the same words by
// any lane of the same wave): the DS instructions of one wave execute in issue
// order, so no lgkmcnt wait is needed, only a compiler fence that keeps the
// accesses in program order.
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

constexpr int NT = 256;
constexpr int T = kWbfmT;
constexpr int M = kWbfmM;
constexpr int Q = kWbfmQ;
using PW = Poly<M, Q, T, NT>;
static_assert(PW::NS == kWbfmNS, "staging size");
constexpr int KP = (PW::NS + 2 * NT - 1) / (2 * NT);  // staged pairs per thread (9)
static_assert(2 * NT * (KP - 1) + 2 * NT - 1 >= PW::NS - 1, "staging coverage");


// ---- front, wave-independent form ----------------------------------------------
// One wave per workgroup and no s_barrier anywhere: every LDS hand-off is inside
// one wave (DS operations of a wave complete in order; wave_lds_fence keeps the
// compiler from reordering around them). Each wave owns a contiguous range of
// decimated outputs [A, B) and walks it in tiles of TW = 64R outputs, one tile's
// 8 TW new inputs prefetched into registers while the previous tile computes.
// Consecutive tiles share 17 polyphase rows (the FIR's Q-row history): they are
// copied inside LDS from the tail to the head of each row, times e^{-j theta NEW}
// so that every tile is NCO-mixed relative to its own origin (the tile's common
// phasor multiplies its outputs, as in the persistent form).
template <int R>
struct Fw {
  static constexpr int TW = 64 * R;      // decimated outputs per tile
  static constexpr int NEW = M * TW;     // inputs entering per tile
  static constexpr int KL = NEW / 128;   // 2-sample loads per lane per tile (4R)
  static constexpr int LR = TW + Q + 2;  // row pitch: rows hold i = 0 .. TW+Q (+1 pad)
  static constexpr int WIN = (R + Q) / 2;  // b128 window reads per lane and phase
  static constexpr int LDS_F2 = M * LR;
  static_assert(LR % 16 == 2, "row pitch = 2 mod 16 (phase-scattered b64 stores)");
  static_assert((R % 2) == 0 && NEW <= kWbfmNS, "phasor table covers the tile");
};


// Lane l receives lane l-1's value; lane 0 receives `first` (DPP wave_shr:1).
__device__ __forceinline__ float wave_shr1(float v, float first) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(first), __float_as_int(v), 0x138,
                                                    0xf, 0xf, false));
}

// Prefetch of a tile's new samples x[B + o], o = 2l + 128k, B = porg + 8Q:
// branch-free 16-B loads at clamped addresses, so the loads stay in flight (a
// branchy prefetch makes the compiler merge register copies behind an s_waitcnt
// vmcnt(0)). Tiles that reach before x[0] or past x[n-1] are re-loaded exactly
// (history / zero padding) at staging time.
// Large inputs (CLAMP = false, n >= 2 NEW): the uniform base is clamped into
// [0, n - NEW], so interior tiles load exactly and one offset register serves
// every load; a boundary tile then loads shifted samples, all of which the
// staging fixup rewrites. Small inputs (CLAMP = true): per-lane clamp of the
// 32-bit offset to [0, n-2] (only the out-of-range samples are wrong).
template <int R, bool A16, bool CLAMP>
__device__ __forceinline__ void front2_load(const f2* __restrict__ x, long long n, long long porg,
                                            int l, f2 (&v)[Fw<R>::KL][2]) {
  const long long B = porg + 8 * Q;
  const f2* __restrict__ xb;
  int lo = 0, hi = 0;
  if constexpr (CLAMP) {
    constexpr long long kSat = 1LL << 30;
    lo = static_cast<int>(max(-B, -kSat));                                   // even
    hi = static_cast<int>(min(max((n - 2 - B) & ~1LL, -kSat), kSat));        // even, >= lo
    xb = x + B;
  } else {
    xb = x + min(max(B, 0LL), (n - Fw<R>::NEW) & ~1LL);
  }
#pragma unroll
  for (int k = 0; k < Fw<R>::KL; ++k) {
    const int o = CLAMP ? min(max(2 * l + 128 * k, lo), hi) : 2 * l + 128 * k;
    if constexpr (A16) {
      // Nontemporal: the input is read once; streaming it past the caches keeps
      // the phi / output lines resident (measured 6.9 vs 6.0 TB/s, membench).
      const f4 w = __builtin_nontemporal_load(reinterpret_cast<const f4*>(xb + o));
      v[k][0] = f2{w.x, w.y};
      v[k][1] = f2{w.z, w.w};
    } else {
      v[k][0] = xb[o];
      v[k][1] = xb[o + 1];
    }
  }
}

// One polyphase phase: window w (b128 pairs of U[c][R l ..]) against taps t.
template <int R>
__device__ __forceinline__ void front2_phase(const f4 (&w)[Fw<R>::WIN], const float (&t)[Q], f2 (&d)[R]) {
#pragma unroll
  for (int h = 0; h < Fw<R>::WIN; ++h) {
    const f2 w0 = f2{w[h].x, w[h].y}, w1 = f2{w[h].z, w[h].w};
    // window entry m -> output rho uses tap q = rho + Q - m
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int q0 = r + Q - 2 * h, q1 = r + Q - 2 * h - 1;
      if (q0 >= 0 && q0 < Q) d[r] = fma2(splat2(t[q0]), w0, d[r]);
      if (q1 >= 0 && q1 < Q) d[r] = fma2(splat2(t[q1]), w1, d[r]);
    }
  }
}

template <int R>
__device__ __forceinline__ void front2_window(const f2* __restrict__ U, int l, int c, f4 (&w)[Fw<R>::WIN]) {
  const f4* row = reinterpret_cast<const f4*>(U + c * Fw<R>::LR + R * l);
#pragma unroll
  for (int h = 0; h < Fw<R>::WIN; ++h) w[h] = row[h];
}
__device__ __forceinline__ void front2_taps(const float* __restrict__ g, int c, float (&t)[Q]) {
#pragma unroll
  for (int q = 0; q < Q; ++q) t[q] = g[c * Q + q];
}

// Polyphase FIR over the 8 phases (rolled: SGPR taps stay at 16 per phase).
template <int R>
__device__ __forceinline__ void front2_decim(const f2* __restrict__ U, int l, const float* __restrict__ g,
                                             f2 (&d)[R]) {
#pragma unroll
  for (int r = 0; r < R; ++r) d[r] = f2{0.0f, 0.0f};
#pragma unroll 1
  for (int c = 0; c < M; ++c) {
    f4 w[Fw<R>::WIN];
    float t[Q];
    front2_window<R>(U, l, c, w);
    front2_taps(g, c, t);
    front2_phase<R>(w, t, d);
  }
}

template <int R, bool A16, bool CLAMP = false>
__global__ __launch_bounds__(64, R <= 2 ? 3 : 2) void k_wbfm_front2(const WbfmArgs a, const WbfmFrontConst C,
                                                    long long L, int wpc) {
  using G = Fw<R>;
  __shared__ __attribute__((aligned(16))) f2 U[G::LDS_F2];
  const int l = threadIdx.x;
  const int ch = blockIdx.x / wpc;
  const long long A = static_cast<long long>(blockIdx.x - ch * wpc) * L;
  const long long B = min(A + L, a.n_dec);
  if (A >= B) return;
  const int ntiles = static_cast<int>((B - A + G::TW) / G::TW);  // outputs A-1 .. B-1

  const f2* __restrict__ tabc = a.tab + static_cast<long long>(ch) * kWbfmNS;
  const bool tiny = a.n < 2;
  const f2* __restrict__ xc = a.x + ch * a.x_stride;
  const f2* __restrict__ xl = tiny ? a.hist_in + ch * kWbfmHist : xc;  // clamp target
  const long long nl = tiny ? kWbfmHist : a.n;
  const f2* __restrict__ hc = a.hist_in + ch * kWbfmHist;
  const uint64_t step = a.step[ch];
  const float* __restrict__ ci = a.carry_in + ch * kWbfmCarry;
  const f2 cprev = f2{ci[4], ci[5]};
  float* __restrict__ phi = a.phi + ch * a.phi_stride;

  // Lane phasors: new samples p = 8Q + 2l + 128k (k < KL) -> e^{j theta p} =
  // tb * tab[128k]; halo samples p = 2l, 2l+1 of the first tile -> tab[p].
  const f4 tv = *reinterpret_cast<const f4*>(tabc + 8 * Q + 2 * l);
  const f2 tb0 = f2{tv.x, tv.y}, tb1 = f2{tv.z, tv.w};
  // Lane phasors e^{j theta p} of the new samples, p = 8Q + 2l + 128k (+1):
  // the same for every tile (each tile is mixed relative to its own origin).
  f2 ph[R <= 2 ? G::KL : 1][2];
  if constexpr (R <= 2) {
#pragma unroll
    for (int k = 0; k < G::KL; ++k) {
      const f2 ek = tabc[128 * k];
      ph[k][0] = cmul(tb0, ek);
      ph[k][1] = cmul(tb1, ek);
    }
  }
  const f2 cn = tabc[G::NEW];
  const f2 corr = f2{cn.x, -cn.y};  // e^{-j theta NEW}
  const int c0 = (-2 * l) & 7, c1 = (-2 * l - 1) & 7;
  const int s0 = c0 * G::LR + (8 * Q + 2 * l + c0) / 8;
  const int s1 = c1 * G::LR + (8 * Q + 2 * l + 1 + c1) / 8;

  long long porg = 8LL * (A - 1 - Q);  // x index of staged sample p = 0
  f2 v[G::KL][2];
  front2_load<R, A16, CLAMP>(xl, nl, porg, l, v);
  {  // halo rows of the first tile (p = 2l, 2l+1), mixed with tab[p]
    const f4 th = *reinterpret_cast<const f4*>(tabc + 2 * l);
    const f2 x0 = load_hist(xc, a.n, hc, kWbfmHist, porg + 2 * l);
    const f2 x1 = load_hist(xc, a.n, hc, kWbfmHist, porg + 2 * l + 1);
    U[c0 * G::LR + (2 * l + c0) / 8] = cmul_rot(x0, f2{th.x, th.y});
    U[c1 * G::LR + (2 * l + 1 + c1) / 8] = cmul_rot(x1, f2{th.z, th.w});
  }

  f2 Sv = f2{1.0f, 0.0f};  // lane m: common phasor of tile nb + m
  int nb = 0;
  f2 carry = f2{0.0f, 0.0f};
  for (int n = 0; n < ntiles; ++n, porg += G::NEW) {
    const long long jd0 = A - 1 + static_cast<long long>(n) * G::TW;
    if (n == nb) {  // tile phasors for the next 64 tiles, one per lane
      Sv = phasor_q64(static_cast<uint64_t>(a.k0 + porg + 1 + static_cast<long long>(l) * G::NEW), step);
      nb += 64;
    }
    // ---- halo: the previous tile's last 17 rows -> rows 0..16 (x e^{-j theta NEW}) ----
    if (n > 0) {
#pragma unroll
      for (int r2 = 0; r2 < 2; ++r2) {
        const int e = l + 64 * r2;
        if (e < 72) {
          const int c = e / 9, h = e - 9 * c;
          const f4 w = *reinterpret_cast<const f4*>(U + c * G::LR + G::TW + 2 * h);
          const f2 y0 = cmul(f2{w.x, w.y}, corr), y1 = cmul(f2{w.z, w.w}, corr);
          *reinterpret_cast<f4*>(U + c * G::LR + 2 * h) = f4{y0.x, y0.y, y1.x, y1.y};
        }
      }
      lds_order();
    }
    // ---- stage the new samples: NCO mix, polyphase scatter ----
    const bool bnd = porg < 0 || porg + 8LL * (G::TW + Q) > a.n;
    if constexpr (R <= 2) {  // lane phasors precomputed once per wave (2 KL registers pairs)
#pragma unroll
      for (int k = 0; k < G::KL; ++k) {
        U[s0 + 16 * k] = cmul_rot_pk(v[k][0], ph[k][0]);
        U[s1 + 16 * k] = cmul_rot_pk(v[k][1], ph[k][1]);
        if (k % 4 == 3) asm volatile("" ::: "memory");  // bound the live temporaries
      }
    } else {
      // Opaque per tile: stops the compiler from hoisting all 2*KL lane phasors
      // tb * tab[128k] out of the tile loop (96 live VGPRs for R = 6).
      int opaque_zero;
      asm volatile("s_mov_b32 %0, 0" : "=s"(opaque_zero));
      const f2* tabk = tabc + opaque_zero;
#pragma unroll
      for (int k = 0; k < G::KL; ++k) {
        const f2 x0 = v[k][0], x1 = v[k][1];
        const f2 ek = tabk[128 * k];
        U[s0 + 16 * k] = cmul_rot_pk(x0, cmul(tb0, ek));
        U[s1 + 16 * k] = cmul_rot_pk(x1, cmul(tb1, ek));
      }
    }
    // ---- prefetch the next tile (lands during this tile's FIR) ----
    // The compiler fence keeps the new loads below the staging stores, so the
    // current and the next tile's registers are never live together.
    asm volatile("" ::: "memory");
    if (n + 1 < ntiles) front2_load<R, A16, CLAMP>(xl, nl, porg + G::NEW, l, v);
    if (bnd) {
      // Tile reaching before x[0] or past x[n-1]: the clamped prefetch staged
      // wrong samples there; rewrite exactly those slots (history / zeros).
      lds_order();
#pragma unroll 1
      for (int p = 8 * Q + l; p < 8 * (G::TW + Q); p += 64) {
        const long long P = porg + p;
        if (!CLAMP || P < 0 || P >= a.n) {  // unclamped loads may be shifted: rewrite all
          const int c = (-p) & 7;
          U[c * G::LR + (p + c) / 8] = cmul_rot(load_hist(xc, a.n, hc, kWbfmHist, P), tabc[p]);
        }
      }
    }
    lds_order();

    // ---- polyphase FIR: outputs jd0 + R l + rho ----
    f2 d[R];
    front2_decim<R>(U, l, C.g, d);
    {
      const int sl = n - (nb - 64);
      const f2 S = f2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(Sv.x), sl)),
                      __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Sv.y), sl))};
#pragma unroll
      for (int r = 0; r < R; ++r) d[r] = cmul(d[r], S);
    }
    if (n == 0 && A == 0 && l == 0) d[0] = cprev;  // d[-1]: carried from the previous call

    // ---- FM discriminator (fm.rs:60-68) ----
    const f2 pv = f2{wave_shr1(d[R - 1].x, carry.x), wave_shr1(d[R - 1].y, carry.y)};
    // Emitted outputs: tile-relative index e = R l + r in [elo, ehi) (32-bit).
    const int elo = static_cast<int>(max(A - jd0, 0LL));
    const int ehi = static_cast<int>(min(B - jd0, static_cast<long long>(G::TW)));
    float* __restrict__ phit = phi + jd0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int e = R * l + r;
      const f2 pr = r == 0 ? pv : d[r - 1];
      if (e >= elo && e < ehi) phit[e] = fm_disc_pk(d[r], pr, C.k);
    }
    carry = f2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(d[R - 1].x), 63)),
               __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d[R - 1].y), 63))};
    // ---- carried state: last decimated sample and raw history ----
    if (jd0 <= a.n_dec - 1 && a.n_dec - 1 < jd0 + G::TW) {
      const int rl = static_cast<int>(a.n_dec - 1 - jd0);
      float* co = a.carry_out + ch * kWbfmCarry;
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (R * l + r == rl) {
          co[4] = d[r].x;
          co[5] = d[r].y;
          co[6] = 0.0f;
          co[7] = 0.0f;
        }
#pragma unroll
      for (int t2 = 0; t2 < kWbfmHist / 64; ++t2) {
        const int t = l + 64 * t2;
        a.hist_out[ch * kWbfmHist + t] = load_hist(xc, a.n, hc, kWbfmHist, a.n - kWbfmHist + t);
      }
    }
  }
}
// ---- back kernel ------------------------------------------------------------
// One workgroup (256 lanes) per block of kBackA = 4096 audio outputs [a0, a0+4096),
// split into two halves 2048 apart. Each half runs LpCascade over its 2048 phi
// plus kBackW = 510 samples of zero-state warm-up (double pole, r = 0.953: the
// transient is < 2e-8 of the state after 510 samples); lane l owns chunk l
// (kBackC = 10 samples) of both halves and runs them as one packed float2
// recurrence (v_pk_* ops: the reference's f32 TDF-II roundings, two chunks at
// once). Chunk states come from an f64 Kogge-Stone scan per half.
// Local index j = i - a0. Half A covers j in [-510, 2050), half B j + 2048.
// Block 0 has no warm-up data: its half-A lanes 0..50 see zero input and lane
// 50's aggregate is replaced by the IIR state carried from the previous call,
// which then enters lane 51 (j = 0) exactly.
// LDS: F (phi, j in [-510, 4098), zero outside [0, n_dec)) for pass 1, aliased
// by P[j] = (f[j], f[j + 2048]) for j in [-124, 2048), the audio FIR's pair image
// (one v_pk_fma_f32 applies a tap to both halves), one pad slot per 8 pairs
// (lane stride 9 pairs = 18 dwords: conflict-free ds_read_b64).
constexpr int kHalf = kBackA / 2;
constexpr int kFSpan = kBackSpan + kHalf;                 // 4608 staged phi
constexpr int kPairs = kHalf + 124;                       // j in [-124, 2048)
__host__ __device__ constexpr int ppos(int e) { return e + (e >> 3); }  // e = j + 124
constexpr int kPDummy = ppos(kPairs) + 1;                 // sink for unneeded warm-up pairs
constexpr int kPSlots = kPDummy + 1;
constexpr int kBackLdsBytes = (kPSlots * 8 > kFSpan * 4 ? kPSlots * 8 : kFSpan * 4);
static_assert(kBackW % kBackC == 0 && 2 * kBackSpan >= kBackA + 2 * kBackW, "back geometry");

// BiquadK::step on two independent streams: identical roundings, packed ops.
struct Biquad2 {
  f2 b0, b1, b2, a1, a2;
  __device__ __forceinline__ f2 step(f2& z1, f2& z2, f2 x) const {
    const f2 y = __builtin_elementwise_fma(x, b0, z1);
    z1 = __builtin_elementwise_fma(x, b1, z2) - a1 * y;
    z2 = x * b2 - a2 * y;
    return y;
  }
  __device__ __forceinline__ f2 lp4(f2 (&s)[4], f2 x) const {
    const f2 y0 = step(s[0], s[1], x);
    return step(s[2], s[3], y0);
  }
};

__global__ __launch_bounds__(NT, 4) void k_wbfm_back(const WbfmArgs a, const WbfmBackConst C) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[kBackLdsBytes];
  __shared__ double tot[4][2][4];
  float* F = reinterpret_cast<float*>(lds);
  f2* P = reinterpret_cast<f2*>(lds);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int ch = blockIdx.y;
  const long long a0 = static_cast<long long>(blockIdx.x) * kBackA;
  const long long a_end = min(a0 + kBackA, a.n_dec);
  const bool first = blockIdx.x == 0;
  const bool last = a_end == a.n_dec;
  const float* __restrict__ phi = a.phi + ch * a.phi_stride;
  const float* __restrict__ ci = a.carry_in + ch * kWbfmCarry;
  const Biquad2 bq{splat2(C.b0), splat2(C.b1), splat2(C.b2), splat2(C.a1), splat2(C.a2)};

  // ---- stage phi (zero outside [0, n_dec)) ----
  for (int e = t; e < kFSpan; e += NT) {
    const long long i = a0 - kBackW + e;
    F[e] = (i >= 0 && i < a.n_dec) ? phi[i] : 0.0f;
  }
  __syncthreads();
  f2 xs[kBackC];  // (half A, half B) inputs of this lane's chunks
#pragma unroll
  for (int i = 0; i < kBackC; i += 2) {  // b64 pairs, 40-B lane stride: conflict-free
    const f2 u = *reinterpret_cast<const f2*>(F + kBackC * t + i);
    const f2 w = *reinterpret_cast<const f2*>(F + kBackC * t + i + kHalf);
    xs[i] = f2{u.x, w.x};
    xs[i + 1] = f2{u.y, w.y};
  }

  // ---- pass 1: zero-state chunk aggregates, f64 scan per half ----
  f2 s[4] = {f2{0, 0}, f2{0, 0}, f2{0, 0}, f2{0, 0}};
#pragma unroll
  for (int i = 0; i < kBackC; ++i) (void)bq.lp4(s, xs[i]);
  double q[2][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    q[0][k] = s[k].x;
    q[1][k] = s[k].y;
  }
  if (first && t == kBackW / kBackC - 1)  // state at j = 0 (previous call) enters lane 51
#pragma unroll
    for (int k = 0; k < 4; ++k) q[0][k] = ci[k];
#pragma unroll 1
  for (int st = 0; st < 6; ++st) {
    const int d = 1 << st;
    double o[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < 4; ++k) o[h][k] = __shfl_up(q[h][k], d, 64);
    if (lane >= d) {
      matvec_acc<4>(C.pw + st * 16, o[0], q[0]);
      matvec_acc<4>(C.pw + st * 16, o[1], q[1]);
    }
  }
  if (lane == 63)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < 4; ++k) tot[wave][h][k] = q[h][k];
  __syncthreads();  // also: every lane holds its inputs (F is dead, P may overwrite it)

  // entering state of this lane's chunks: lanemats[lane] * (state entering the
  // wave) + the exclusive in-wave prefix
  f2 ef[4];
  {
    double cw[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    for (int w = 0; w < wave; ++w) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        double vv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) vv[k] = tot[w][h][k];
        matvec_acc<4>(C.mw, cw[h], vv);
#pragma unroll
        for (int k = 0; k < 4; ++k) cw[h][k] = vv[k];
      }
    }
    double e[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double o = __shfl_up(q[h][k], 1, 64);
        e[h][k] = lane == 0 ? 0.0 : o;
      }
    matvec_acc<4>(a.lanemats + lane * 16, cw[0], e[0]);
    matvec_acc<4>(a.lanemats + lane * 16, cw[1], e[1]);
#pragma unroll
    for (int k = 0; k < 4; ++k) ef[k] = f2{static_cast<float>(e[0][k]), static_cast<float>(e[1][k])};
  }

  // ---- pass 2: the reference's f32 recurrence from the entering state ----
  // Pairs j < -124 (warm-up not needed by the FIR) and, in block 0, j < 0 (the
  // previous call's f values are written below) go to a dummy slot.
  const int jlo = first ? 0 : -124;
  const int j0 = kBackC * t - kBackW;
  if (!last) {
#pragma unroll
    for (int i = 0; i < kBackC; ++i) {
      const int j = j0 + i;
      const f2 f = bq.lp4(ef, xs[i]);
      P[j >= jlo ? ppos(j + 124) : kPDummy] = f;
    }
  } else {
    // last block: also capture the IIR state after sample n_dec - 1
    const int jl = static_cast<int>(a.n_dec - 1 - a0);  // local index of the last sample
    float cap[4] = {0, 0, 0, 0};
    bool have = false;
#pragma unroll
    for (int i = 0; i < kBackC; ++i) {
      const int j = j0 + i;
      const f2 f = bq.lp4(ef, xs[i]);
      P[j >= jlo ? ppos(j + 124) : kPDummy] = f;
      if (j == jl && jl < kHalf) {  // half A owns j < 2048 (its tail past 2048 is B's)
#pragma unroll
        for (int k = 0; k < 4; ++k) cap[k] = ef[k].x;
        have = true;
      }
      if (j + kHalf == jl && j >= 0) {  // half B owns j >= 2048 (its warm-up is A's)
#pragma unroll
        for (int k = 0; k < 4; ++k) cap[k] = ef[k].y;
        have = true;
      }
    }
    if (have) {
      float* co = a.carry_out + ch * kWbfmCarry;
#pragma unroll
      for (int k = 0; k < 4; ++k) co[k] = cap[k];
    }
  }
  // Pairs j in [-124, 0): .y = f[j + 2048] came from half B's warm-up; the exact
  // value is half A's (converged) f at 1924 .. 2047. Block 0: .x = f[-124 .. -1]
  // of the previous call.
  __syncthreads();
  if (t < 124) {
    P[ppos(t)].y = P[ppos(t + kHalf)].x;
    if (first) P[ppos(t)].x = ci[8 + 4 + t];
  }
  __syncthreads();

  // ---- audio FIR (fir.rs:57-66, quirk-mapped taps) ----
  // Lane t owns outputs j = 8t + i and j + 2048 (i < 8) as float2 pairs. Output
  // j, tap k = 16 kb + kk reads f[j - k]: window index m = i + 15 - kk of the
  // 23 pairs starting at e = 8t - 16kb - 15 + 124 = 8(t - 2kb) + 109; with
  // ppos, slot = 9(t - 2kb) + 109 + m + ((109 + m) >> 3): a per-lane base plus
  // compile-time offsets.
  {
    constexpr int R = 8, KA = 128;
    f2 acc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = f2{0.0f, 0.0f};
#pragma unroll 1
    for (int kb = 0; kb < KA / 16; ++kb) {
      const f2* __restrict__ Pl = P + 9 * (t - 2 * kb) + 109;
      f2 w[R + 15];
#pragma unroll
      for (int m = 0; m < R + 15; ++m) w[m] = Pl[m + ((109 + m) >> 3)];
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const f2 tap = splat2(C.a[16 * kb + kk]);
#pragma unroll
        for (int i = 0; i < R; ++i) acc[i] = fma2(tap, w[i + 15 - kk], acc[i]);
      }
    }
    float* __restrict__ y = a.y + ch * a.y_stride + a0;
    const int nv = static_cast<int>(a_end - a0);
    if (nv == kBackA) {
      float4* ya = reinterpret_cast<float4*>(y + R * t);
      float4* yb = reinterpret_cast<float4*>(y + kHalf + R * t);
      if ((reinterpret_cast<uintptr_t>(y) & 15) == 0) {
        ya[0] = float4{acc[0].x, acc[1].x, acc[2].x, acc[3].x};
        ya[1] = float4{acc[4].x, acc[5].x, acc[6].x, acc[7].x};
        yb[0] = float4{acc[0].y, acc[1].y, acc[2].y, acc[3].y};
        yb[1] = float4{acc[4].y, acc[5].y, acc[6].y, acc[7].y};
      } else {
#pragma unroll
        for (int i = 0; i < R; ++i) {
          y[R * t + i] = acc[i].x;
          y[kHalf + R * t + i] = acc[i].y;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int j = R * t + i;
        if (j < nv) y[j] = acc[i].x;
        if (j + kHalf < nv) y[j + kHalf] = acc[i].y;
      }
    }
  }
  if (last && t < 128) {  // last 128 f values (fhist of the next call)
    const int j = static_cast<int>(a.n_dec - 128 + t - a0);
    float f;
    if (j >= 0) f = j < kHalf ? P[ppos(j + 124)].x : P[ppos(j - kHalf + 124)].y;
    else f = j >= -124 ? P[ppos(j + 124)].x : ci[8 + 128 + j];  // reaches into the carried history
    a.carry_out[ch * kWbfmCarry + 8 + t] = f;
  }
}

namespace fu {
using G = Fw<2>;
// debug timing: lane 0 records s_memrealtime (100 MHz) at phase boundaries
__device__ __forceinline__ void trace(const WbfmArgs& a, int r, int point) {
  if (a.trace && (threadIdx.x & 63) == 0)
    a.trace[static_cast<long long>(r) * kFuTracePoints + point] =
        static_cast<long long>(__builtin_amdgcn_s_memrealtime());
}
constexpr int PB = kFuTail;  // FIR history pairs (j >= -128)

template <int N>
struct Geo {
  static constexpr int L = 128 * N;           // outputs per sub-range
  static constexpr int NH = L / 2;            // per IIR half
  static constexpr int CH = NH / 64;          // IIR chunk per lane per half = FIR outputs per lane per half
  static_assert((CH & (CH - 1)) == 0 && CH >= 8, "chunk a power of two");
  // FIR pair slots: one pad per CH pairs -> lane stride CH+1 pairs (2(CH+1) dwords:
  // 2 x odd, so the ds_read_b64 of 32 lanes hit distinct bank pairs)
  __host__ __device__ static constexpr int pslot(int e) { return e + e / CH; }
  static constexpr int PSlots = pslot(NH + PB) + 1;
};

__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// This wave's stores have completed (reached the agent coherence point).
__device__ __forceinline__ void stores_done() { __builtin_amdgcn_s_waitcnt(0x0F70); }
__device__ __forceinline__ void publish(uint32_t* flag, uint32_t epoch, int l) {
  stores_done();
  if (l == 0) st_agent(flag, epoch);
}
// Bounded wait for a flag holding `epoch`: at most `spin` polls (spin == 0: time
// out at once without looking; test-only). On timeout the handle's error word
// (host-visible, see Block::dev_err) is set and the wave continues, so the kernel
// always drains; the host reports the error at its next check of the handle.
__device__ __forceinline__ void wait_for(const uint32_t* flag, uint32_t epoch, int* err, uint32_t spin) {
  for (uint32_t it = 0; it < spin; ++it) {
    if (ld_agent(flag) == epoch) {
      asm volatile("" ::: "memory");
      return;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double u2d(uint32_t lo, uint32_t hi) {
  return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}
}  // namespace fu

// One front tile (tiles aligned at the segment start). The registers v hold this
// tile's prefetched inputs on entry; on exit they hold the loads issued for the
// next tile (pf), possibly a dummy L2-resident tile past the segment.
struct FuTile {
  const WbfmArgs& a;
  const WbfmFrontConst& C;
  f2* U;
  float* Phi;
  const float* Gt;  // decimator taps in LDS (phase-major)
  const f2* xc;
  const f2* hc;
  const f2* tabc;
  int ch, l, s0, s1;
  f2 corr;
  bool first;  // the channel's first range: d[A-1] is the carried sample
};
struct FuPrefetch {  // where the next prefetched tile starts
  const f2* xl;
  long long nl, porg;
  bool on;
};

// ---- front tile, four-group decimator ---------------------------------------------
// The polyphase FIR with EIGHT outputs per lane. The 64 lanes are the four
// ds_read_b128 lane groups of gfx950 (A = {0-3, 12-15, 20-27}, B = {4-11, 16-19,
// 28-31}, C, D = A, B + 32); group g sums phases 2g and 2g+1 for outputs 8l'..8l'+7
// (l' = l & 15), and two permlane swaps (rows 0<->1, 2<->3, then the halves) add the
// four partial sums, leaving every lane two outputs. Per lane and tile: 24 window + 8
// tap ds_read_b128 and eight independent FMA chains per phase. Image rows carry one
// 16-B pad after every four chunks, so lane windows start 5 chunks apart and the 16
// lanes of a read group hit 16 distinct bank quads; the pitch (91 chunks, odd)
// spreads the phase-scattered b64 staging stores.
namespace g8 {
constexpr int PCH = 91;          // row pitch, 16-B chunks
constexpr int LRS = 2 * PCH;     // row pitch, f2 slots
constexpr int LDS_F2 = M * LRS;  // 11648 B
__host__ __device__ constexpr int pchunk(int c) { return 5 * (c >> 2) + (c & 3); }
__host__ __device__ constexpr int slot(int i) { return 2 * pchunk(i >> 1) + (i & 1); }
static_assert(slot(fu::G::TW + Q) < LRS && pchunk(fu::G::TW / 2) == 80, "row geometry");
__device__ __forceinline__ int group(int l) {
  const int i = l & 31;
  const bool a = i < 4 || (i >= 12 && i < 16) || (i >= 20 && i < 28);
  return (l >> 5) * 2 + (a ? 0 : 1);
}
// the lane holding the output before this lane's first one (lane 0: the carry)
__device__ __forceinline__ int prev_lane(int l) {
  const int row = l >> 4, lp = l & 15;
  return row == 0 ? 47 + lp : row == 2 ? lp : row == 1 ? 32 + lp : 16 + lp;
}
// this lane's first output (tile-relative): rows 0, 2, 1, 3 own 8l' + {0,1}, {2,3}, {4,5}, {6,7}
__device__ __forceinline__ int first_out(int l) {
  const int row = l >> 4;
  return 8 * (l & 15) + 2 * (row == 0 ? 0 : row == 2 ? 1 : row == 1 ? 2 : 3);
}
// One phase c of a lane's eight outputs: 12 window + 4 tap ds_read_b128 and 128
// v_pk_fma_f32. FIRST: the chains start with a product (d need not be zeroed).
// ORD: taps read first and the taps walked from q = Q-1 down, so the first FMAs
// need only the first window reads (entries 1..8) rather than the last.
template <bool FIRST, bool ORD>
__device__ __forceinline__ void phase(const f2* __restrict__ U, int c, int lp, const float* __restrict__ Gt,
                                      f2 (&d)[8]) {
  const f4* __restrict__ row = reinterpret_cast<const f4*>(U + c * LRS) + 5 * lp;
  const f4* __restrict__ tq = reinterpret_cast<const f4*>(Gt + c * Q);
  f4 w[12];
  float t[Q];
  if constexpr (ORD) {
#pragma unroll
    for (int q4 = Q / 4 - 1; q4 >= 0; --q4) {
      const f4 u = tq[q4];
      t[4 * q4] = u.x;
      t[4 * q4 + 1] = u.y;
      t[4 * q4 + 2] = u.z;
      t[4 * q4 + 3] = u.w;
    }
#pragma unroll
    for (int h = 0; h < 12; ++h) w[h] = row[5 * (h >> 2) + (h & 3)];
  } else {
#pragma unroll
    for (int h = 0; h < 12; ++h) w[h] = row[5 * (h >> 2) + (h & 3)];
#pragma unroll
    for (int q4 = 0; q4 < Q / 4; ++q4) {
      const f4 u = tq[q4];
      t[4 * q4] = u.x;
      t[4 * q4 + 1] = u.y;
      t[4 * q4 + 2] = u.z;
      t[4 * q4 + 3] = u.w;
    }
  }
#pragma unroll
  for (int qi = 0; qi < Q; ++qi) {
    const int q = ORD ? Q - 1 - qi : qi;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int m = r + Q - q;  // window entry 1 .. 23 (tap q of output 8l' + r)
      const f4& wc = w[m >> 1];
      const f2 xv = (m & 1) ? f2{wc.z, wc.w} : f2{wc.x, wc.y};
      if (FIRST && qi == 0) {
        d[r] = splat2(t[q]) * xv;
      } else {
        d[r] = fma2(splat2(t[q]), xv, d[r]);
      }
    }
  }
}
}  // namespace g8

template <bool A16, bool CLAMP>
__device__ __forceinline__ void fu_tile8(const FuTile& T, int n, long long porg, long long jd0,
                                         const f2 (&ph)[8][2], f2 (&v)[8][2], const FuPrefetch& pf, f2 Sv,
                                         f2& carry, float* __restrict__ phit, int svi) {
  using G = fu::G;
  f2* __restrict__ U = T.U;
  const int l = T.l;
  // Halo (n > 0): the previous tile's entries TW .. TW+Q of each row become entries
  // 0 .. Q, times e^{-j theta NEW}. Entries 0..15 of every row (lane l: row l & 7,
  // pair l >> 3: conflict-free b128 stores) and entry Q of rows 1..7 (lanes 0..6;
  // row 0's entry Q is a staged sample). The sources are read BEFORE the staging
  // stores overwrite them and written after (DS operations of a wave execute in
  // order), so the read's latency hides behind the staging.
  const int hc = l & 7, hh = l >> 3;
  f4 hw = f4{0, 0, 0, 0};
  f2 hq = f2{0, 0};
  if (n > 0) {
    hw = *reinterpret_cast<const f4*>(U + hc * g8::LRS + 2 * (80 + g8::pchunk(hh)));
    if (l < 7) hq = U[(l + 1) * g8::LRS + g8::slot(G::TW + Q)];
  }
  const bool bnd = porg < 0 || porg + 8LL * (G::TW + Q) > T.a.n;
#pragma unroll
  for (int k = 0; k < G::KL; ++k) {  // entry i + 16k = slot(i) + 20k
    U[T.s0 + 20 * k] = cmul_rot_pk(v[k][0], ph[k][0]);
    U[T.s1 + 20 * k] = cmul_rot_pk(v[k][1], ph[k][1]);
    if (k % 4 == 3) asm volatile("" ::: "memory");
  }
  asm volatile("" ::: "memory");
  if (n > 0) {
    const f2 y0 = cmul(f2{hw.x, hw.y}, T.corr), y1 = cmul(f2{hw.z, hw.w}, T.corr);
    *reinterpret_cast<f4*>(U + hc * g8::LRS + 2 * g8::pchunk(hh)) = f4{y0.x, y0.y, y1.x, y1.y};
    if (l < 7) U[(l + 1) * g8::LRS + g8::slot(Q)] = cmul(hq, T.corr);
  }
  // unconditional: a conditional prefetch makes the compiler's wait counting assume
  // the loads may be absent and drain them (vmcnt(0))
  front2_load<2, A16, CLAMP>(pf.xl, pf.nl, pf.porg, l, v);
  if (bnd) {
    lds_order();
#pragma unroll 1
    for (int p = (n == 0 ? 0 : 8 * Q) + l; p < 8 * (G::TW + Q); p += 64) {
      const long long Pp = porg + p;
      if (!CLAMP || Pp < 0 || Pp >= T.a.n || p < 8 * Q) {
        const int c = (-p) & 7;
        U[c * g8::LRS + g8::slot((p + c) / 8)] = cmul_rot(load_hist(T.xc, T.a.n, T.hc, kWbfmHist, Pp), T.tabc[p]);
      }
    }
  }
  lds_order();
  // group g: phases 2g, 2g+1; window entries 8l' .. 8l'+23 of the phase's row
  const int g = g8::group(l), lp = l & 15;
  f2 d[8];
  // phase 2g opens the eight chains with a product (no zeroing), phase 2g+1 follows;
  // the compiler barrier keeps the second phase's reads behind the first's FMAs
  // (both windows live at once would cost 48 more VGPRs)
  g8::phase<true, true>(U, 2 * g, lp, T.Gt, d);
  asm volatile("" ::: "memory");
  g8::phase<false, true>(U, 2 * g + 1, lp, T.Gt, d);
  // rows 0<->1, 2<->3: even rows keep outputs 0..3, odd rows 4..7 (x: d[i], y: d[i+4])
  f2 K[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const auto sx = __builtin_amdgcn_permlane16_swap(__float_as_uint(d[i].x), __float_as_uint(d[i + 4].x), false, false);
    const auto sy = __builtin_amdgcn_permlane16_swap(__float_as_uint(d[i].y), __float_as_uint(d[i + 4].y), false, false);
    K[i] = f2{__uint_as_float(sx[0]), __uint_as_float(sy[0])} + f2{__uint_as_float(sx[1]), __uint_as_float(sy[1])};
  }
  // halves: rows 0, 1 keep K[0..1], rows 2, 3 K[2..3]
  f2 F[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const auto sx = __builtin_amdgcn_permlane32_swap(__float_as_uint(K[i].x), __float_as_uint(K[i + 2].x), false, false);
    const auto sy = __builtin_amdgcn_permlane32_swap(__float_as_uint(K[i].y), __float_as_uint(K[i + 2].y), false, false);
    F[i] = f2{__uint_as_float(sx[0]), __uint_as_float(sy[0])} + f2{__uint_as_float(sx[1]), __uint_as_float(sy[1])};
  }
  const f2 S = f2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(Sv.x), svi)),
                  __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Sv.y), svi))};
  F[0] = cmul(F[0], S);
  F[1] = cmul(F[1], S);
  if (n == 0 && !T.first) {
    // d[A-1], the previous segment's last output, from this tile's image (rows
    // i = 0..15; the segment setup staged U[c][0], c >= 1): taps 2l, 2l+1 per
    // lane, summed over the wave
    f2 acc = f2{0.0f, 0.0f};
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const int k = 2 * l + t2, c = k & 7, q = k >> 3;
      acc = fma2(splat2(T.Gt[c * Q + q]), U[c * g8::LRS + g8::slot(15 - q)], acc);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
      acc += f2{__shfl_xor(acc.x, off, 64), __shfl_xor(acc.y, off, 64)};
    carry = cmul(acc, S);
  }
  // (an LDS permute: the lane-swap form, permlane32 + permlane16 + DPP, measured
  // 4-5 us slower per launch)
  const int src = g8::prev_lane(l);
  f2 pv = f2{__shfl(F[1].x, src, 64), __shfl(F[1].y, src, 64)};
  if (l == 0) pv = carry;
  const int j0 = g8::first_out(l);
  *reinterpret_cast<f2*>(phit + j0) = f2{fm_disc_pk_rcp(F[0], pv, T.C.k), fm_disc_pk_rcp(F[1], F[0], T.C.k)};
  carry = f2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(F[1].x), 63)),
             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(F[1].y), 63))};
  const WbfmArgs& a = T.a;
  if (jd0 <= a.n_dec - 1 && a.n_dec - 1 < jd0 + G::TW) {  // carried state of the next call
    const int rl = static_cast<int>(a.n_dec - 1 - jd0);
    float* co = a.carry_out + T.ch * kWbfmCarry;
#pragma unroll
    for (int r = 0; r < 2; ++r)
      if (j0 + r == rl) {
        co[4] = F[r].x;
        co[5] = F[r].y;
        co[6] = 0.0f;
        co[7] = 0.0f;
      }
#pragma unroll
    for (int t2 = 0; t2 < kWbfmHist / 64; ++t2) {
      const int t = l + 64 * t2;
      a.hist_out[T.ch * kWbfmHist + t] = load_hist(T.xc, a.n, T.hc, kWbfmHist, a.n - kWbfmHist + t);
    }
  }
}

// Segment geometry.
struct FuRange {
  int r, ch, wl;
  long long A, B;
  int Lr;
  bool first, last;
};
// Where segment g's first tile starts.
__device__ __forceinline__ FuPrefetch fu_origin(const WbfmArgs& a, const FuRange& g) {
  const bool tiny = a.n < 2;
  FuPrefetch p;
  p.xl = tiny ? a.hist_in + g.ch * kWbfmHist : a.x + g.ch * a.x_stride;
  p.nl = tiny ? kWbfmHist : a.n;
  p.porg = 8LL * (g.A - Q);
  p.on = true;
  return p;
}

// ---- segmented chain: k_wbfm_seg -----------------------------------------------------
// One round of waves (the grid is the resident capacity); each wave owns a segment of
// a channel, whole sub-ranges of kSgL = 1024 decimated outputs (8 front tiles):
//   * every sub-range's 8 tiles leave 1024 phi in LDS; then its back runs: iir16
//     (LpCascade from the exact entering state), the reference's f32 recurrence
//     into the audio FIR's pair image, the 125-tap audio FIR, the stores;
//   * a segment's first sub-range needs the state at the END of the previous
//     segment. It runs its zero-state pass only (zs_only16: its end state and last
//     128 IIR outputs are the true ones to f32 resolution, as the host checks
//     ||A^896|| < 1e-10), parks its 1024 phi in its global slot and continues;
//   * each segment publishes its end state and last 128 IIR outputs (agent-scope
//     stores + flag) as soon as its last sub-range's IIR is done; at its end it
//     waits for its predecessor's record (bounded: a timeout sets the handle's
//     device error word, which the host reports) and runs the first sub-range's back.
//     A record is published before its writer waits, so no wait chain forms, and
//     the predecessor is the previous blockIdx, dispatched before the waiter: a wait
//     always ends, whatever other streams hold on the chip.
// Issue priority: a SIMD's arbiter favours the older of its two waves; the later-
// dispatched wave takes s_setprio 1 for the first 9/16 of its tiles, the earlier
// one for the rest, so both finish together.
constexpr int kSegPrioQ16 = 9;  // the later wave of a SIMD leads for 9/16 of its tiles (measured A/B)
namespace sg {
constexpr int NS = 8;          // front tiles per sub-range
using Y = fu::Geo<NS>;         // L 1024, NH 512, CH 8
constexpr int L = Y::L;
constexpr int CH = Y::CH;
constexpr int WBytes = (Y::PSlots * 8 > L * 4) ? Y::PSlots * 8 : L * 4;
constexpr int kSegSlot = kSeg4Slot;  // u32 words: end-state record, then sub-range 0's phi

__device__ __forceinline__ double uni(double v) {  // wave-uniform value -> SGPRs
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane(static_cast<int>(b));
  const int hi = __builtin_amdgcn_readfirstlane(static_cast<int>(b >> 32));
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// Sub-range IIR with lane l owning the 16 CONSECUTIVE samples 16l .. 16l+15: chunk E
// (16l .. 16l+7) in the x halves and chunk O (16l+8 .. 16l+15) in the y halves of
// xs, both zero-state passes packed. The lane aggregate A^8 zE + zO is scanned over
// the 64 lanes (Kogge-Stone, f64, step matrices A^(16 2^s) = pw[s+1], mh) with the
// entering state sw folded into lane 0, so the scan yields every lane's TRUE entering
// state directly: no per-lane transition matrices (lanemats) and half the f64 work
// of zero_state + the A^{CH l} products. ef: the f32 entering states of E and O;
// send: the f64 end state after sample L-1 (uniform).
// The step matrices, read with scalar loads (constant address space) at each use: held in
// SGPRs across the segment loop they were spilled to VGPR lanes and re-read by v_readlane
// (VALU work), ~200 per sub-range.
typedef const __attribute__((address_space(4))) double* cmat_t;
__device__ __forceinline__ cmat_t mats_of(const WbfmFusedConst& Bc) {
  const double* p = Bc.mats;
  asm volatile("" : "+s"(p));  // opaque per back: no hoisting of the loads out of the segment loop
  return (cmat_t)(p);  // C-style: generic -> constant address space
}
template <int S>
__device__ __forceinline__ void matvec_c(cmat_t M, const double (&x)[S], double (&y)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i)
#pragma unroll
    for (int j = 0; j < S; ++j) y[i] = __builtin_fma(M[i * S + j], x[j], y[i]);
}
__device__ __forceinline__ void iir16(const WbfmFusedConst& Bc, const float* __restrict__ Phi, int l,
                                      const double (&sw)[4], f2 (&xs)[CH], f2 (&ef)[4], double (&send)[4]) {
#pragma unroll
  for (int i = 0; i < CH; i += 4) {
    const f4 u = *reinterpret_cast<const f4*>(Phi + 16 * l + i);
    const f4 w = *reinterpret_cast<const f4*>(Phi + 16 * l + 8 + i);
    xs[i] = f2{u.x, w.x};
    xs[i + 1] = f2{u.y, w.y};
    xs[i + 2] = f2{u.z, w.z};
    xs[i + 3] = f2{u.w, w.w};
  }
  lds_order();
  const Biquad2 bq{splat2(Bc.b0), splat2(Bc.b1), splat2(Bc.b2), splat2(Bc.a1), splat2(Bc.a2)};
  f2 z[4] = {f2{0, 0}, f2{0, 0}, f2{0, 0}, f2{0, 0}};
#pragma unroll
  for (int i = 0; i < CH; ++i) (void)bq.lp4(z, xs[i]);
  double zE[4], q[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    zE[k] = z[k].x;
    q[k] = z[k].y;
  }
  const cmat_t pw = mats_of(Bc);
  matvec_c<4>(pw, zE, q);  // A^8 zE + zO
  {
    double f[4] = {0, 0, 0, 0};
    matvec_c<4>(pw + 16, sw, f);  // A^16 sw
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] += l == 0 ? f[k] : 0.0;
  }
#pragma unroll 1
  for (int st = 0; st < 6; ++st) {
    const int dd = 1 << st;
    double o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = __shfl_up(q[k], dd, 64);
    if (l >= dd) matvec_c<4>(pw + (st + 1) * 16, o, q);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long long b = __double_as_longlong(q[k]);
    const int lo = __builtin_amdgcn_readlane(static_cast<int>(b), 63);
    const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), 63);
    send[k] = __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
  }
  double eE[4], eO[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double o = __shfl_up(q[k], 1, 64);
    eE[k] = l == 0 ? sw[k] : o;
    eO[k] = zE[k];
  }
  matvec_c<4>(pw, eE, eO);  // entering O = A^8 (entering E) + zE
#pragma unroll
  for (int k = 0; k < 4; ++k) ef[k] = f2{static_cast<float>(eE[k]), static_cast<float>(eO[k])};
}

// zs_only with iir16: sub-range 0's zero-state end state sw and zero-state last 128
// IIR outputs (lanes 56..63 run their pass 2; tmp: 128 floats of free LDS).
__device__ __forceinline__ void zs_only16(const WbfmFusedConst& Bc, const float* Phi, float* tmp, int l,
                                          double (&sw)[4], float (&hout)[2]) {
  const double zero[4] = {0, 0, 0, 0};
  f2 xs[CH], ef[4];
  iir16(Bc, Phi, l, zero, xs, ef, sw);
  const Biquad2 bq{splat2(Bc.b0), splat2(Bc.b1), splat2(Bc.b2), splat2(Bc.a1), splat2(Bc.a2)};
  int to = 16 * (l - 56);
  asm volatile("" : "+v"(to));  // not hoisted and spilled (see iir16's pass 2)
  float* __restrict__ tl = tmp + to;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const f2 f = bq.lp4(ef, xs[i]);
    if (l >= 56) {  // f[16l + i], f[16l + 8 + i]: tail index 16(l - 56) + i (+ 8)
      tl[i] = f.x;
      tl[8 + i] = f.y;
    }
  }
  lds_order();
  hout[0] = tmp[l];
  hout[1] = tmp[l + 64];
  lds_order();
}

// ---- audio FIR on the matrix cores ---------------------------------------------------
// y[o] = sum_k a[k] f[o - k] (fir.rs:57-66, quirk-mapped taps, k < 128) as Toeplitz
// products on v_mfma_f32_16x16x32_f16: group g of 256 outputs o = 256 g + 16 J + I
// (I the row, J the column), K = 160 window entries kap of the column's window
// f[256 g + 16 J - 128 + kap]: A[I][kap] = a[I + 128 - kap] (zero outside [0, 128)),
// B[kap][J] = the window. f16 parts: f 2^sf = fh + fl, a 2^st = ah + al, three products
// ah fh + ah fl + al fh per step, accumulated in f32. st is the host's (WbfmFusedConst
// tscale = 2^-st: max |a| 2^st in [2^14, 2^15)); sf is chosen PER SUB-RANGE from the max
// |f| over its window (its 1024 outputs and the 128 history values): max |f| 2^sf in
// [2^14, 2^15), so fh keeps 11 significant bits at every signal level and fl 11 more
// (relative error of each product ~3 2^-24, an f32 FMA chain's order; tools/micro/
// mfma_fir.hip) - a fixed scale from the worst-case bound lost bits on quiet audio
// (VERDICT r4 weak 1a). The history carried to the next sub-range, segment or call is
// the exact f32 f (Tx), never the f16 reconstruction. The A fragments (5 steps x hi/lo
// x 64 lanes x 8 halves) come from global memory (WbfmArgs.afrag, L2-resident).
// f planes in LDS: index e = j + 128 for j in [-128, 1040), padded 8 halves per 128
// (pe: the 16 column reads of one ds_read_b128 hit distinct banks).
__host__ __device__ constexpr int pe(int e) { return e + ((e >> 7) << 3); }
constexpr int kFpN = pe(128 + 1024 + 16) + 8;  // halves per plane
#ifndef ORION_WBFM_EXACT_FIR
#define ORION_WBFM_EXACT_FIR 0
#endif
#if ORION_WBFM_EXACT_FIR
// Build option (make DEFS=-DORION_WBFM_EXACT_FIR=1): the audio FIR on
// v_mfma_f32_16x16x4_f32, exact f32 operands and an FMA chain per output: one f32 plane,
// 4 pad floats per 64 (the 16 columns x 4 k of a read hit distinct banks), taps
// At[m] = a[m - 31] (host). Measured round 6: +21 us per C2 launch, and the chain's
// error against the oracle unchanged to three digits at every signal level
// (profiles/r6_wbfm_ab_f32fir.txt), so the split-f16 form stays the default.
__host__ __device__ constexpr int pf(int e) { return e + 4 * (e >> 6); }
constexpr int kTxOff = pf(128 + 1024 + 16) * 4;
#else
constexpr int kTxOff = 2 * kFpN * 2;           // bytes: the exact next history (128 f32) after the planes
#endif
static_assert(kTxOff % 16 == 0 && kTxOff + 128 * 4 <= WBytes, "f planes + exact history fit the sub-range region");
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ _Float16 hi16(float x) { return static_cast<_Float16>(x); }
__device__ __forceinline__ _Float16 lo16(float x, _Float16 h) { return static_cast<_Float16>(x - static_cast<float>(h)); }

// Max over the wave of a non-negative v (DPP within rows, then the row swaps); every
// lane gets the result.
template <int CTRL>
__device__ __forceinline__ float dpp_max(float v) {
  return fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false)));
}
__device__ __forceinline__ float wave_max(float v) {
  v = dpp_max<0xB1>(v);   // quad_perm [1,0,3,2]
  v = dpp_max<0x4E>(v);   // quad_perm [2,3,0,1]
  v = dpp_max<0x141>(v);  // row_half_mirror: the two quads of a half-row
  v = dpp_max<0x140>(v);  // row_mirror: the two half-rows
  const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r16[0]), __uint_as_float(r16[1]));
  const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r32[0]), __uint_as_float(r32[1]));
}

// The back of one sub-range [A0, A0 + Lr) from its exact entering state sw and
// FIR history hist (f[A0 - 128 + l + 64 r], exact f32): pass 2 (the reference's f32
// recurrence) -> f planes -> audio FIR -> y. Returns the end state (after
// f[A0 + L - 1]) in sw and this sub-range's last 128 IIR outputs in hist (exact). The
// planes alias Phi (Phi is read into registers first). chan_last: the channel's last
// sub-range (writes the IIR state and FIR history carried to the next call).
// publish_r >= 0: publish the end state and last 128 IIR outputs to the successor
// (publish_end) as soon as they are known, before the audio FIR.
// Publish a segment's end state and last 128 IIR outputs to its successor.
__device__ __forceinline__ void publish_end(const WbfmArgs& a, int r, const double (&sw)[4], const float (&hist)[2],
                                            int l) {
  uint32_t* slot = a.hand + static_cast<long long>(r) * kSegSlot;
  if (l < 8) {
    const int kk = l >> 1;
    const double v8 = kk == 0 ? sw[0] : kk == 1 ? sw[1] : kk == 2 ? sw[2] : sw[3];
    const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v8));
    fu::st_agent(slot + 2 + l, (l & 1) ? static_cast<uint32_t>(b >> 32) : static_cast<uint32_t>(b));
  }
  fu::st_agent(slot + 16 + l, __float_as_uint(hist[0]));
  fu::st_agent(slot + 16 + 64 + l, __float_as_uint(hist[1]));
  fu::publish(a.flags + 3LL * r, a.epoch, l);
}

__device__ __forceinline__ void back(const WbfmArgs& a, const WbfmFusedConst& Bc, int ch, long long A0, int Lr,
                                     bool chan_last, const float* Phi, void* Pv, const uint32_t* __restrict__ Aw,
                                     int l, double (&sw)[4], float (&hist)[2], int publish_r = -1,
                                     int trace_r = -1) {
  const Biquad2 bq{splat2(Bc.b0), splat2(Bc.b1), splat2(Bc.b2), splat2(Bc.a1), splat2(Bc.a2)};
  _Float16* __restrict__ Fh = static_cast<_Float16*>(Pv);
  _Float16* __restrict__ Fl = Fh + kFpN;
  float* __restrict__ Tx = reinterpret_cast<float*>(static_cast<unsigned char*>(Pv) + kTxOff);
  f2 xs[CH];
  {  // lane l: samples 16l .. 16l+15 (iir16); f replaces x in xs (zeros past Lr)
    f2 ef[4];
    double send[4];
    iir16(Bc, Phi, l, sw, xs, ef, send);
    if (trace_r >= 0) fu::trace(a, trace_r, 10);
    const int jl = Lr - 1;
    float cap[4] = {0, 0, 0, 0};
    bool have = false;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int j = 16 * l + i;  // and j + 8
      const f2 f = bq.lp4(ef, xs[i]);
      xs[i] = f2{j < Lr ? f.x : 0.0f, j + 8 < Lr ? f.y : 0.0f};
      const int te = j - Lr + 128;  // index in the next history f[Lr - 128 + t]
      if (te >= 0 && te < 128) Tx[te] = f.x;
      if (te + 8 >= 0 && te + 8 < 128) Tx[te + 8] = f.y;
      if (chan_last) {
        if (j == jl) {
#pragma unroll
          for (int k = 0; k < 4; ++k) cap[k] = ef[k].x;
          have = true;
        }
        if (j + 8 == jl) {
#pragma unroll
          for (int k = 0; k < 4; ++k) cap[k] = ef[k].y;
          have = true;
        }
      }
    }
    if (have) {
      float* co = a.carry_out + ch * kWbfmCarry;
#pragma unroll
      for (int k = 0; k < 4; ++k) co[k] = cap[k];
    }
    // the state after f[Lr - 1] (Lr < L: a multiple of 16 unless it is the channel's end)
    const int lend = Lr >= L ? 63 : max(0, (Lr >> 4) - 1);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      sw[k] = static_cast<double>(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(ef[k].y), lend)));
  }
  if (Lr < 128) {  // short sub-range: the old history's tail stays history
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      const int t = l + 64 * r2 - Lr;
      if (t >= 0) Tx[t] = hist[r2];
    }
  }
#if ORION_WBFM_EXACT_FIR
  const int sf = 0;
  {
    float* __restrict__ Fp = static_cast<float*>(Pv);
    const int e0 = pf(128 + 16 * l);
    *reinterpret_cast<f4*>(Fp + e0) = f4{xs[0].x, xs[1].x, xs[2].x, xs[3].x};
    *reinterpret_cast<f4*>(Fp + e0 + 4) = f4{xs[4].x, xs[5].x, xs[6].x, xs[7].x};
    *reinterpret_cast<f4*>(Fp + e0 + 8) = f4{xs[0].y, xs[1].y, xs[2].y, xs[3].y};
    *reinterpret_cast<f4*>(Fp + e0 + 12) = f4{xs[4].y, xs[5].y, xs[6].y, xs[7].y};
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) Fp[pf(l + 64 * r2)] = hist[r2];
    if (l < 4) *reinterpret_cast<f4*>(Fp + pf(128 + 1024 + 4 * l)) = f4{0, 0, 0, 0};
  }
#else
  // this sub-range's f scale: max |f| over the FIR's window (outputs and history)
  float mx = fmaxf(fabsf(hist[0]), fabsf(hist[1]));
#pragma unroll
  for (int i = 0; i < CH; ++i) mx = fmaxf(mx, fmaxf(fabsf(xs[i].x), fabsf(xs[i].y)));
  mx = wave_max(mx);
  const int sf = __builtin_amdgcn_readfirstlane(min(100, 15 - __builtin_amdgcn_frexp_expf(mx)));  // mx 2^sf < 2^15
  {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const int e0 = pe(128 + 16 * l);  // 16 consecutive halves, inside one 128-run
#pragma unroll
    for (int i = 0; i < CH; i += 2) {
      h2 eh, el, oh, ol;  // f16 parts of f[16l + i] (E) and f[16l + 8 + i] (O), two at a time
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float fe = __builtin_amdgcn_ldexpf(xs[i + u].x, sf), fo = __builtin_amdgcn_ldexpf(xs[i + u].y, sf);
        eh[u] = hi16(fe);
        el[u] = lo16(fe, eh[u]);
        oh[u] = hi16(fo);
        ol[u] = lo16(fo, oh[u]);
      }
      *reinterpret_cast<h2*>(Fh + e0 + i) = eh;
      *reinterpret_cast<h2*>(Fl + e0 + i) = el;
      *reinterpret_cast<h2*>(Fh + e0 + 8 + i) = oh;
      *reinterpret_cast<h2*>(Fl + e0 + 8 + i) = ol;
    }
  }
#pragma unroll
  for (int r2 = 0; r2 < 2; ++r2) {  // j in [-128, 0): the history
    const int e = pe(l + 64 * r2);
    const float x = __builtin_amdgcn_ldexpf(hist[r2], sf);
    const _Float16 h = hi16(x);
    Fh[e] = h;
    Fl[e] = lo16(x, h);
  }
  if (l < 2) {  // j in [1024, 1040): read by the last columns' windows against zero taps
    const h8 z = h8{0, 0, 0, 0, 0, 0, 0, 0};
    *reinterpret_cast<h8*>(Fh + pe(128 + 1024 + 8 * l)) = z;
    *reinterpret_cast<h8*>(Fl + pe(128 + 1024 + 8 * l)) = z;
  }
#endif
  lds_order();
#pragma unroll
  for (int r2 = 0; r2 < 2; ++r2) hist[r2] = Tx[l + 64 * r2];  // f[Lr - 128 + t]: the next history
  if (publish_r >= 0) publish_end(a, publish_r, sw, hist, l);
  if (chan_last) {  // the next call's FIR history: f[n_dec - 128 .. n_dec)
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) a.carry_out[ch * kWbfmCarry + 8 + l + 64 * r2] = hist[r2];
  }
  if (trace_r >= 0) fu::trace(a, trace_r, 11);  // debug: IIR done
  {
    const int J = l & 15, kg = l >> 4;
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
    // per K-step: the A fragments (8 consecutive reversed taps r[kap0 - I - 1 ..], four
    // aligned words of the parity copy, LDS) and the eight plane reads issued together,
    // then the four groups' MFMAs interleaved (independent accumulators back to back).
    // (The fragments from global memory, L2-resident, cost ~0.5 us per step under the
    // fronts' HBM load: the trace's FIR phase, round 6.)
#if ORION_WBFM_EXACT_FIR
    {
      const float* __restrict__ Fp = static_cast<const float*>(Pv);
      const float* __restrict__ At = reinterpret_cast<const float*>(Aw);
      const int I = l & 15;
#pragma unroll 4
      for (int st = 0; st < 40; ++st) {
        const float av = At[I - 4 * st - kg + 159];
        const int p = pf(16 * J + 4 * st + kg);
        float b[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) b[g] = Fp[p + 272 * g];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b[g], acc[g], 0, 0, 0);
      }
    }
#else
    const int I = l & 15;
#pragma unroll 1
    for (int st = 0; st < 5; ++st) {
      h8 ah, al;
      {
        const int o = 32 * st + 8 * kg - I - 1, p = o & 1;
        const uint32_t* wh = Aw + p * kAudTapWords + ((o + 16 + p) >> 1);
        const uint32_t* wl = wh + 2 * kAudTapWords;
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const u4 vh = u4{wh[0], wh[1], wh[2], wh[3]}, vl = u4{wl[0], wl[1], wl[2], wl[3]};
        ah = __builtin_bit_cast(h8, vh);
        al = __builtin_bit_cast(h8, vl);
      }
      h8 bh[4], bl[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int e = pe(256 * g + 16 * J + 32 * st + 8 * kg);
        bh[g] = *reinterpret_cast<const h8*>(Fh + e);
        bl[g] = *reinterpret_cast<const h8*>(Fl + e);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[g], acc[g], 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[g], acc[g], 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[g], acc[g], 0, 0, 0);
      asm volatile("" ::: "memory");  // the next step's plane reads stay behind these MFMAs (registers)
      if (trace_r >= 0 && st == 0) fu::trace(a, trace_r, 13);  // debug: step 0's operands arrived, MFMAs issued
    }
#endif
    if (trace_r >= 0) fu::trace(a, trace_r, 14);  // debug: every MFMA issued
    // lane (J, kg) holds outputs 256 g + 16 J + 4 kg + r, r < 4
    float* __restrict__ y = a.y + ch * a.y_stride + A0;
    const float ys = __builtin_amdgcn_ldexpf(Bc.tscale, -sf);  // 2^-(sf + st)
    if (Lr == L && (reinterpret_cast<uintptr_t>(y) & 15) == 0) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(y + 256 * g + 16 * J + 4 * kg) =
            float4{acc[g][0] * ys, acc[g][1] * ys, acc[g][2] * ys, acc[g][3] * ys};
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = 256 * g + 16 * J + 4 * kg + r;
          if (j < Lr) y[j] = acc[g][r] * ys;
        }
    }
  }
  lds_order();
  if (trace_r >= 0) fu::trace(a, trace_r, 12);  // debug: audio FIR done (stores issued)
}

}  // namespace sg

template <bool A16, bool CLAMP>
__global__ __launch_bounds__(64, 2) void k_wbfm_seg(const WbfmArgs a, const WbfmFrontConst C,
                                                    const WbfmFusedConst Bc, int spc, int S) {
  using G = fu::G;
  constexpr int TW = G::TW;
  __shared__ __attribute__((aligned(16))) f2 U[g8::LDS_F2];
  __shared__ __attribute__((aligned(16))) unsigned char wreg[sg::WBytes];
  __shared__ __attribute__((aligned(16))) float Gt[128];
  __shared__ __attribute__((aligned(16))) uint32_t Aw[kAudFragBytes / 4];  // audio FIR taps (sg::back)
  float* Phi = reinterpret_cast<float*>(wreg);
  f2* P = reinterpret_cast<f2*>(wreg);
  const int l = threadIdx.x & 63;
  Gt[l] = C.g[l];
  Gt[l + 64] = C.g[l + 64];
  {
    const uint32_t* __restrict__ aw = static_cast<const uint32_t*>(a.afrag);
#pragma unroll
    for (int i = 0; i < kAudFragBytes / 4 / 64; ++i) Aw[l + 64 * i] = aw[l + 64 * i];
  }
  FuRange g;
  // Segment r = blockIdx.x: a segment's predecessor (whose end state it waits for) has
  // the smaller blockIdx, so it was dispatched first whatever else holds the CUs (an
  // XCD-contiguous map measured within noise, -0.8 us, and made seven segments wait on
  // the last-dispatched blocks: VERDICT r3 weak 5).
  g.r = blockIdx.x;
  g.ch = g.r / spc;
  g.wl = g.r - g.ch * spc;
  g.A = static_cast<long long>(g.wl) * S;
  g.B = min(g.A + S, a.n_dec);
  g.Lr = static_cast<int>(g.B - g.A);
  g.first = g.wl == 0;
  g.last = g.B == a.n_dec;
  const bool late = blockIdx.x >= (gridDim.x >> 1);
  const int nsub = (g.Lr + sg::L - 1) / sg::L;
  const int ntiles = nsub * sg::NS;
  uint32_t* const myslot = a.hand + static_cast<long long>(g.r) * sg::kSegSlot;
  fu::trace(a, g.r, 0);

  // One tile of inputs in flight (32 VGPRs; two tiles left the kernel spilling).
  const FuPrefetch org = fu_origin(a, g);
  f2 va[G::KL][2];
  front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg, l, va);
  const f2* __restrict__ tabc = a.tab + static_cast<long long>(g.ch) * kWbfmNS;
  const f2* __restrict__ xc = a.x + g.ch * a.x_stride;
  const f2* __restrict__ hc = a.hist_in + g.ch * kWbfmHist;
  const f2 cn = tabc[G::NEW];
  const int c0 = (-2 * l) & 7, c1 = (-2 * l - 1) & 7;
  const FuTile T{a, C, U, Phi, Gt, xc, hc, tabc, g.ch, l, c0 * g8::LRS + g8::slot((8 * Q + 2 * l + c0) / 8),
                 c1 * g8::LRS + g8::slot((8 * Q + 2 * l + 1 + c1) / 8), f2{cn.x, -cn.y}, g.first};
  long long porg = org.porg;
  {  // halo rows of the first tile (clamped here, exact via the boundary fixup)
    const long long P0 = porg + 2 * l;
    const long long hi = (org.nl & ~1LL) - 2;
    const long long Pc = P0 < 0 ? 0 : (P0 > hi ? hi : P0);
    const f2 x0 = org.xl[Pc], x1 = org.xl[Pc + 1];
    const f4 th = *reinterpret_cast<const f4*>(tabc + 2 * l);
    U[c0 * g8::LRS + g8::slot((2 * l + c0) / 8)] = cmul_rot(x0, f2{th.x, th.y});
    U[c1 * g8::LRS + g8::slot((2 * l + 1 + c1) / 8)] = cmul_rot(x1, f2{th.z, th.w});
  }
  {  // p = -l (row c = l, entry 0), l = 1..7: used only by d[A-1]. Not the first
     // segment, so porg - l >= 0: a plain load (a branchy one would drain the prefetch)
    const long long Pm = max(porg - (l & 7), 0LL);
    const f2 xm = xc[Pm];
    const f2 tc = tabc[l & 7];
    if (!g.first && l >= 1 && l < 8) U[l * g8::LRS] = cmul_rot(xm, f2{tc.x, -tc.y});
  }
  f2 Sv = f2{0, 0};
  f2 carry = f2{0.0f, 0.0f};
  if (g.first) {  // d[-1]: the last decimated sample of the previous call (fm.rs:29 on reset)
    const float* ci = a.carry_in + g.ch * kWbfmCarry;
    carry = f2{ci[4], ci[5]};
  }
  double sw[4] = {0, 0, 0, 0};  // IIR state entering the next sub-range
  float hist[2] = {0, 0};       // its FIR history
  // past the segment: a dummy read of the channel's first tile, shared by every
  // segment of the channel so that it hits in L2
  const FuPrefetch dummy{org.xl, org.nl, -8LL * Q, true};

#pragma unroll 1
  for (int sub = 0, n = 0; sub < nsub; ++sub) {
    // per-lane staging phasors e^{j theta p}, p = 8Q + 2l + r + 128k: rebuilt per
    // sub-range so that they are dead (not holding 32 VGPRs) during a back
    f2 ph[G::KL][2];
    {
      const f4 tv = *reinterpret_cast<const f4*>(tabc + 8 * Q + 2 * l);
      const f2 tb0 = f2{tv.x, tv.y}, tb1 = f2{tv.z, tv.w};
#pragma unroll
      for (int k = 0; k < G::KL; ++k) {
        const f2 ek = tabc[128 * k];
        ph[k][0] = cmul(tb0, ek);
        ph[k][1] = cmul(tb1, ek);
      }
    }
    const long long A0 = g.A + static_cast<long long>(sub) * sg::L;
    const int Lr = static_cast<int>(min(static_cast<long long>(sg::L), g.B - A0));
#pragma unroll 1
    for (int tin = 0; tin < sg::NS; ++tin, ++n, porg += G::NEW) {
      if ((16 * n < kSegPrioQ16 * ntiles) == late) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
      if ((n & 63) == 0)  // lane l: the common phasor of tile n + l
        Sv = phasor_q64(static_cast<uint64_t>(a.k0 + porg + 1 + static_cast<long long>(l) * G::NEW),
                        a.step[g.ch]);
      const long long jd0 = g.A + static_cast<long long>(n) * TW;
      const FuPrefetch p0 = n + 1 < ntiles ? FuPrefetch{org.xl, org.nl, porg + G::NEW, true} : dummy;
      fu_tile8<A16, CLAMP>(T, n, porg, jd0, ph, va, p0, Sv, carry, Phi + TW * tin, n & 63);
    }
    lds_order();
    if (sub == 0) {
      // keep sub-range 0's phi for the deferred back in the segment's global slot
      f4* gs = reinterpret_cast<f4*>(myslot + kFuSlot);
#pragma unroll
      for (int i = 0; i < sg::L / 256; ++i) gs[l + 64 * i] = *reinterpret_cast<const f4*>(Phi + 4 * (l + 64 * i));
      sg::zs_only16(Bc, Phi, Phi, l, sw, hist);
      if (nsub == 1 && !g.last) sg::publish_end(a, g.r, sw, hist, l);
    } else {
      const bool lastsub = sub == nsub - 1;
      if (sub <= 3) fu::trace(a, g.r, 3 + sub);
      sg::back(a, Bc, g.ch, A0, Lr, g.last && lastsub, Phi, P, Aw, l, sw, hist, lastsub && !g.last ? g.r : -1,
               sub == 1 ? g.r : -1);
      if (sub <= 3) fu::trace(a, g.r, 6 + sub);
    }
  }
  fu::trace(a, g.r, 1);
  // ---- deferred: sub-range 0 from the predecessor's end state ----
  // The parked phi's loads are issued first and written to LDS after the predecessor's
  // record has arrived, so that their round trip overlaps the flag poll's.
  const f4* gs = reinterpret_cast<const f4*>(myslot + kFuSlot);
  f4 u[sg::L / 256];
#pragma unroll
  for (int i = 0; i < sg::L / 256; ++i) u[i] = __builtin_nontemporal_load(gs + l + 64 * i);
  if (g.first) {
    const float* __restrict__ ci = a.carry_in + g.ch * kWbfmCarry;
#pragma unroll
    for (int k = 0; k < 4; ++k) sw[k] = ci[k];
    hist[0] = ci[8 + l];
    hist[1] = ci[8 + 64 + l];
  } else {
    fu::wait_for(a.flags + 3LL * (g.r - 1), a.epoch, a.err, a.spin);
    const uint32_t* ps = a.hand + static_cast<long long>(g.r - 1) * sg::kSegSlot;
#pragma unroll
    for (int k = 0; k < 4; ++k) sw[k] = sg::uni(fu::u2d(fu::ld_agent(ps + 2 + 2 * k), fu::ld_agent(ps + 3 + 2 * k)));
    hist[0] = __uint_as_float(fu::ld_agent(ps + 16 + l));
    hist[1] = __uint_as_float(fu::ld_agent(ps + 16 + 64 + l));
  }
#pragma unroll
  for (int i = 0; i < sg::L / 256; ++i) *reinterpret_cast<f4*>(Phi + 4 * (l + 64 * i)) = u[i];
  lds_order();
  fu::trace(a, g.r, 2);
  sg::back(a, Bc, g.ch, g.A, min(sg::L, g.Lr), g.last && nsub == 1, Phi, P, Aw, l, sw, hist);
  fu::trace(a, g.r, 3);
}

}  // namespace

namespace {

constexpr int kFrontR = 2;

// Wave ranges for the two-kernel path's front: as many resident waves as LDS and
// registers allow, rounded down to a multiple of 4 per CU (one per SIMD each, so
// no SIMD carries more waves than another), one round; each wave owns N tiles =
// N*TW - 1 phi outputs.
struct Front2Plan {
  int grid, wpc;
  long long L;
};
template <int R>
Front2Plan front2_plan(long long n_dec, int nch, int ncu) {
  using G = Fw<R>;
  int per_cu = std::min<int>((160 * 1024) / static_cast<int>(G::LDS_F2 * sizeof(f2)), R <= 2 ? 12 : 8);
  per_cu = std::max(4, per_cu & ~3);
  const long long slots = static_cast<long long>(per_cu) * ncu;
  const long long tiles = static_cast<long long>(nch) * ((n_dec + G::TW) / G::TW);
  const long long N = std::max<long long>(1, (tiles + slots - 1) / slots);
  Front2Plan p;
  p.L = N * G::TW - 1;
  p.wpc = static_cast<int>((n_dec + p.L - 1) / p.L);
  p.grid = p.wpc * nch;
  return p;
}

template <int R>
void launch_front2(bool a16, long long n_dec, int nch, int ncu, const WbfmArgs& a,
                   const WbfmFrontConst& f, hipStream_t s) {
  const Front2Plan fp = front2_plan<R>(n_dec, nch, ncu);
  if (a.n < 2LL * Fw<R>::NEW) {  // small input: per-lane clamped loads
    if (a16) k_wbfm_front2<R, true, true><<<fp.grid, 64, 0, s>>>(a, f, fp.L, fp.wpc);
    else k_wbfm_front2<R, false, true><<<fp.grid, 64, 0, s>>>(a, f, fp.L, fp.wpc);
  } else {
    if (a16) k_wbfm_front2<R, true><<<fp.grid, 64, 0, s>>>(a, f, fp.L, fp.wpc);
    else k_wbfm_front2<R, false><<<fp.grid, 64, 0, s>>>(a, f, fp.L, fp.wpc);
  }
}

}  // namespace

long long wbfm_seg_slots(long long n_dec, int nch) {
  return static_cast<long long>(nch) * ((n_dec + kSgL - 1) / kSgL) + 1;
}

// One round: as many segments as resident waves (per channel: the channel's share,
// at least one sub-range per segment), each a whole number of sub-ranges.
void launch_wbfm_seg(const WbfmArgs& a, const WbfmFrontConst& f, const WbfmFusedConst& b, int nch,
                     int max_segments, hipStream_t s) {
  static_assert(sg::L == kSgL, "sub-range geometry");
  if (a.n_dec <= 0 || nch <= 0) return;
  const int cap = resident_per_cu(reinterpret_cast<const void*>(k_wbfm_seg<true, false>), 64) * device_cus();
  // max_segments > 0: that many segments, also beyond one round of resident waves: every
  // segment waits only on the previous blockIdx, dispatched before it, so a grid of
  // several rounds cannot deadlock (later rounds start as earlier segments retire)
  const long long capx = max_segments > 0 ? max_segments : cap;
  const long long nsub_ch = (a.n_dec + kSgL - 1) / kSgL;
  long long spc = std::max<long long>(1, std::min<long long>(capx / nch, nsub_ch));
  const long long S = (nsub_ch + spc - 1) / spc * kSgL;
  spc = (a.n_dec + S - 1) / S;
  const long long grid = spc * nch;
  if (grid > (1LL << 31) - 1 || S > (1LL << 30)) throw HipError("WBFM segment geometry out of range");
  const bool a16 = (reinterpret_cast<uintptr_t>(a.x) % 16 == 0) && (a.x_stride % 2 == 0);
  const bool clamp = a.n < 2LL * Fw<2>::NEW;
  const int gi = static_cast<int>(grid), sp = static_cast<int>(spc), Si = static_cast<int>(S);
  if (clamp) {
    if (a16) k_wbfm_seg<true, true><<<gi, 64, 0, s>>>(a, f, b, sp, Si);
    else k_wbfm_seg<false, true><<<gi, 64, 0, s>>>(a, f, b, sp, Si);
  } else {
    if (a16) k_wbfm_seg<true, false><<<gi, 64, 0, s>>>(a, f, b, sp, Si);
    else k_wbfm_seg<false, false><<<gi, 64, 0, s>>>(a, f, b, sp, Si);
  }
  ORION_LAUNCH_CHECK();
}

void launch_wbfm(const WbfmArgs& a, const WbfmFrontConst& f, const WbfmBackConst& b, int nch,
                 hipStream_t s) {
  if (a.n_dec <= 0 || nch <= 0) return;
  const int ncu = device_cus();
  const bool a16 = (reinterpret_cast<uintptr_t>(a.x) % 16 == 0) && (a.x_stride % 2 == 0);
  const dim3 gb(div_up(a.n_dec, kBackA), nch);
  launch_front2<kFrontR>(a16, a.n_dec, nch, ncu, a, f, s);
  k_wbfm_back<<<gb, NT, 0, s>>>(a, b);
  ORION_LAUNCH_CHECK();
}

}  // namespace orion
