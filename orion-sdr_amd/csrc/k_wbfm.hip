// k_wbfm.hip — the WBFM demodulation chain on gfx950 (the north-star path).
//
// Reference composition (docs/demodulate.md:128-133, SURVEY §3 stack 2):
//   Rotator(-f_off).rotate_block (dsp/rotator.rs:74-85)
//   -> FirDecimator(fs, 8, ...)  (dsp/decim.rs:44-76; kept outputs only here)
//   -> FmQuadratureDemod         (demodulate/fm.rs:45-77: discriminator + LpCascade)
//   -> FirLowpass                (dsp/fir.rs:47-66, the audio filter).
//
// k_wbfm_front — persistent: 4 workgroups (256 lanes) per CU, each streaming a
//   contiguous range of tiles (one XCD owns one contiguous eighth, so the
//   120-sample halo a tile shares with its neighbour is an L2 hit). Per tile of
//   512 decimated outputs: the 4224 cf32 inputs were prefetched into registers
//   (16-B loads) during the previous tile; they are NCO-mixed with a per-position
//   phasor table (registers) and scattered into the polyphase LDS image, the
//   next tile's loads are issued, and the polyphase FIR runs at the kept outputs
//   (two per lane, packed FMA, taps from SGPRs). The tile's common phasor factor
//   multiplies the 512 decimated outputs; the discriminator (atan2_approx op for
//   op) produces 511 phi values (tiles overlap by one decimated sample).
// k_wbfm_back — one workgroup per 4096 audio outputs: LpCascade over phi by a
//   state-carry scan (19 samples per lane, f64 Kogge-Stone + cross-wave carry,
//   re-run with the reference's f32 TDF-II update), started 768 samples early
//   from a zero state (pole radius 0.953: the transient is < 1e-8 of the state
//   after 641 samples); then the 125-tap audio FIR, register-blocked and packed.
// The first tile / workgroup of each channel starts from the exact state carried
// from the previous call (last decimated sample, 128 raw inputs, IIR state, last
// 128 IIR outputs), so k calls equal one call on the concatenation.
#include "iir.hpp"
#include "kernels.hpp"
#include "poly.hpp"

namespace orion {
namespace {

constexpr int NT = 256;
constexpr int T = kWbfmT;
constexpr int M = kWbfmM;
constexpr int Q = kWbfmQ;
using PW = Poly<M, Q, T, NT>;
static_assert(PW::NS == kWbfmNS, "staging size");
constexpr int KP = (PW::NS + 2 * NT - 1) / (2 * NT);  // staged pairs per thread (9)
static_assert(2 * NT * (KP - 1) + 2 * NT - 1 >= PW::NS - 1, "staging coverage");

__device__ __forceinline__ float lp4_step(const BiquadK& bq, float (&s)[4], float x) {
  const float y0 = bq.step(s[0], s[1], x);
  return bq.step(s[2], s[3], y0);
}

// Prefetch of one tile's inputs: branch-free 16-B loads at clamped addresses, so
// the loads stay in flight (a branchy prefetch makes the compiler merge register
// copies behind an s_waitcnt vmcnt(0)). Tiles that reach before x[0] or past
// x[n-1] are re-loaded exactly (history / zero padding) at staging time.
template <bool A16>
__device__ __forceinline__ void front_load(const WbfmArgs& a, int ch, long long porg, int t,
                                           f2 (&v)[KP][2]) {
  const bool tiny = a.n < 2;  // nothing safe to clamp into: read the history buffer
  const f2* __restrict__ x = tiny ? a.hist_in : a.x + ch * a.x_stride;
  const long long hi = (tiny ? kWbfmHist : (a.n & ~1LL)) - 2;
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const int p = 2 * t + 2 * NT * k;
    if (p < PW::NS) {
      long long P = porg + p;
      P = P < 0 ? 0 : (P > hi ? hi : P);
      if constexpr (A16) {
        const f4 w = *reinterpret_cast<const f4*>(x + P);
        v[k][0] = f2{w.x, w.y};
        v[k][1] = f2{w.z, w.w};
      } else {
        v[k][0] = x[P];
        v[k][1] = x[P + 1];
      }
    }
  }
}

__device__ __forceinline__ bool front_boundary(const WbfmArgs& a, long long porg) {
  return porg < 0 || porg + PW::NS > a.n;
}

template <bool A16>
__global__ __launch_bounds__(NT, 4) void k_wbfm_front(const WbfmArgs a, const WbfmFrontConst C,
                                                      int tiles_per_ch, int nch) {
  __shared__ __attribute__((aligned(16))) f2 U[PW::LDS_F2];
  __shared__ __attribute__((aligned(16))) f2 D[T];
  const int t = threadIdx.x;
  // Tile range of this workgroup: XCD (blockIdx % 8) owns a contiguous eighth of
  // the (channel, tile) space; its G/8 workgroups interleave through it.
  const int total = tiles_per_ch * nch;
  const int g8 = gridDim.x >> 3;
  const int per = (total + 7) >> 3;
  const int lo = (blockIdx.x & 7) * per;
  const int hi = min(lo + per, total);
  // Staging slots of this thread: p = 2t + 512k, p+1; the phase c is the same
  // for every k (512 = 0 mod 8), so slot(p + 512k) = slot(p) + 64k.
  const int s0 = PW::slot(2 * t), s1 = PW::slot(2 * t + 1);

  f2 v[KP][2];
  f2 tb0 = f2{1.0f, 0.0f}, tb1 = f2{1.0f, 0.0f};  // e^{j theta 2t}, e^{j theta (2t+1)}
  const f2* __restrict__ tabc = a.tab;
  uint64_t step = 0;
  f2 cprev = f2{1.0f, 0.0f};
  int cur_ch = -1;
  int u = lo + static_cast<int>(blockIdx.x >> 3);
  if (u < hi) {
    const int ch = u / tiles_per_ch;
    const long long Jd = static_cast<long long>(u - ch * tiles_per_ch) * kWbfmPhi - 1;
    front_load<A16>(a, ch, static_cast<long long>(M) * (Jd - Q), t, v);
  }
  for (; u < hi; u += g8) {
    const int ch = u / tiles_per_ch;
    const int b = u - ch * tiles_per_ch;
    const long long J = static_cast<long long>(b) * kWbfmPhi;  // first phi of this tile
    const long long Jd = J - 1;                                 // first decimated output
    const long long porg = static_cast<long long>(M) * (Jd - Q);
    if (ch != cur_ch) {  // per-channel constants, loaded before any prefetch is in flight
      tabc = a.tab + static_cast<long long>(ch) * PW::NS;
      const f4 tv = *reinterpret_cast<const f4*>(tabc + 2 * t);
      tb0 = f2{tv.x, tv.y};
      tb1 = f2{tv.z, tv.w};
      step = a.step[ch];
      const float* ci = a.carry_in + ch * kWbfmCarry;
      cprev = f2{ci[4], ci[5]};  // d[-1]: the last decimated sample of the previous call
      cur_ch = ch;
    }
    // ---- stage: NCO mix, polyphase scatter ----
    // e^{j theta (2t + 512k)} = e^{j theta 2t} * e^{j theta 512k}; the second
    // factor is uniform (scalar loads of tab[512k]). A boundary tile (before x[0]
    // or past x[n-1]) replaces the clamped prefetch by the exact samples.
    const bool bnd = front_boundary(a, porg);
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const int p = 2 * t + 2 * NT * k;
      if (p < PW::NS) {
        f2 x0 = v[k][0], x1 = v[k][1];
        if (bnd) {
          const f2* __restrict__ xc = a.x + ch * a.x_stride;
          const f2* __restrict__ hc = a.hist_in + ch * kWbfmHist;
          x0 = load_hist(xc, a.n, hc, kWbfmHist, porg + p);
          x1 = load_hist(xc, a.n, hc, kWbfmHist, porg + p + 1);
        }
        const f2 ek = tabc[2 * NT * k];
        U[s0 + 64 * k] = cmul_rot(x0, cmul(tb0, ek));
        U[s1 + 64 * k] = cmul_rot(x1, cmul(tb1, ek));
      }
    }
    // ---- prefetch the next tile (lands during this tile's compute) ----
    {
      const int un = u + g8;
      if (un < hi) {
        const int chn = un / tiles_per_ch;
        const long long Jdn = static_cast<long long>(un - chn * tiles_per_ch) * kWbfmPhi - 1;
        front_load<A16>(a, chn, static_cast<long long>(M) * (Jdn - Q), t, v);
      }
    }
    lds_barrier();  // LDS-only: the prefetch stays in flight

    // ---- polyphase FIR at the kept outputs; common phasor of the tile ----
    {
      f2 acc[PW::R];
      PW::compute(U, t, [&](int c, int q) { return C.g[c * Q + q]; }, acc);
      const f2 S = phasor_q64(static_cast<uint64_t>(a.k0 + porg + 1), step);
      D[2 * t] = cmul(acc[0], S);
      D[2 * t + 1] = cmul(acc[1], S);
      if (b == 0 && t == 0) D[0] = cprev;
    }
    lds_barrier();

    // ---- FM discriminator (fm.rs:60-68) ----
    float* __restrict__ phi = a.phi + ch * a.phi_stride;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = 2 * t + r;
      const long long j = J + i;
      if (i < kWbfmPhi && j < a.n_dec) phi[j] = fm_disc(D[i + 1], D[i], C.k);
    }
    // ---- carried state: last decimated sample and raw history ----
    if (J <= a.n_dec - 1 && a.n_dec - 1 < J + kWbfmPhi) {
      float* co = a.carry_out + ch * kWbfmCarry;
      if (t == 0) {
        const f2 last = D[a.n_dec - 1 - Jd];
        co[4] = last.x;
        co[5] = last.y;
        co[6] = 0.0f;
        co[7] = 0.0f;
      }
      if (t < kWbfmHist)
        a.hist_out[ch * kWbfmHist + t] =
            load_hist(a.x + ch * a.x_stride, a.n, a.hist_in + ch * kWbfmHist, kWbfmHist, a.n - kWbfmHist + t);
    }
  }
}

// ---- back kernel LDS images ---------------------------------------------------
// F: phi staging, local sample l = 0 .. kBackSpan-1 (plain; read once by the IIR).
// P: audio-FIR window pairs P[l] = (f[l], f[l + 2048]) for l = -128 .. 2815, one
//    pad slot every 8 pairs (lane stride 8 -> 18 dwords: ds_read_b64 conflict-free).
//    P aliases F: F is dead once every lane holds its IIR inputs in registers.
constexpr int kHalf = kBackA / 2;
constexpr int kPairs = kBackSpan - kBackA + kHalf + 128;  // 2944
__device__ __forceinline__ int ppos(int l) { return (l + 128) + ((l + 128) >> 3); }
constexpr int kPSlots = kPairs + kPairs / 8 + 8;
constexpr int kBackLdsBytes = (kPSlots * 8 > kBackSpan * 4 ? kPSlots * 8 : kBackSpan * 4);

__device__ __forceinline__ void put_f(f2* P, int l, float f) {
  if (l < kPairs - 128) P[ppos(l)].x = f;
  if (l >= kHalf - 128) P[ppos(l - kHalf)].y = f;
}
__device__ __forceinline__ float get_f(const f2* P, int l) {
  return l < kPairs - 128 ? P[ppos(l)].x : P[ppos(l - kHalf)].y;
}

__global__ __launch_bounds__(NT) void k_wbfm_back(const WbfmArgs a, const WbfmBackConst C) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[kBackLdsBytes];
  __shared__ double tot[4][4];
  float* F = reinterpret_cast<float*>(lds);
  f2* P = reinterpret_cast<f2*>(lds);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int ch = blockIdx.y;
  const long long a0 = static_cast<long long>(blockIdx.x) * kBackA;
  const long long a_end = min(a0 + kBackA, a.n_dec);
  long long js = a0 - (kBackSpan - kBackA);
  const bool first = js <= 0;
  if (first) js = 0;
  const int cnt = static_cast<int>(a_end - js);
  const float* __restrict__ phi = a.phi + ch * a.phi_stride;
  const float* __restrict__ ci = a.carry_in + ch * kWbfmCarry;
  const BiquadK bq{C.b0, C.b1, C.b2, C.a1, C.a2};

  for (int i = t; i < cnt; i += NT) F[i] = phi[js + i];
  __syncthreads();

  // ---- LpCascade: lane chunk [19 t, 19 t + 19) ----
  float xs[kBackC];
#pragma unroll
  for (int i = 0; i < kBackC; ++i) xs[i] = F[kBackC * t + i];  // stride 19: conflict-free
  float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int i = 0; i < kBackC; ++i)
    if (kBackC * t + i < cnt) (void)lp4_step(bq, s, xs[i]);
  double q[4] = {s[0], s[1], s[2], s[3]};
  wave_scan_inclusive<4>(q, C.pw, lane);
  if (lane == 63)
#pragma unroll
    for (int i = 0; i < 4; ++i) tot[wave][i] = q[i];
  __syncthreads();  // also: every lane has read its xs (F is dead, P may overwrite it)
  double cw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) cw[i] = first ? static_cast<double>(ci[i]) : 0.0;
  for (int w = 0; w < wave; ++w) {
    double vv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) vv[i] = tot[w][i];
    matvec_acc<4>(C.mw, cw, vv);
#pragma unroll
    for (int i = 0; i < 4; ++i) cw[i] = vv[i];
  }
  double e[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double o = __shfl_up(q[i], 1, 64);
    e[i] = lane == 0 ? 0.0 : o;
  }
  matvec_acc<4>(a.lanemats + lane * 16, cw, e);
  float ef[4] = {static_cast<float>(e[0]), static_cast<float>(e[1]), static_cast<float>(e[2]),
                 static_cast<float>(e[3])};
  if (first && t < 128) put_f(P, t - 128, ci[8 + t]);  // f[-128 .. -1] from the previous call
#pragma unroll
  for (int i = 0; i < kBackC; ++i) {
    const int li = kBackC * t + i;
    if (li < cnt) put_f(P, li, lp4_step(bq, ef, xs[i]));
  }
  const bool last = a_end == a.n_dec;
  if (last && kBackC * t <= cnt - 1 && cnt - 1 < kBackC * t + kBackC) {
    float* co = a.carry_out + ch * kWbfmCarry;
#pragma unroll
    for (int i = 0; i < 4; ++i) co[i] = ef[i];
  }
  __syncthreads();

  // ---- audio FIR (fir.rs:57-66, quirk-mapped taps) over [a0, a_end) ----
  // Lane t owns outputs a0 + 8t + i and a0 + 2048 + 8t + i (i < 8) as float2
  // pairs: one ds_read_b64 fetches (f[l], f[l+2048]), one v_pk_fma_f32 applies a
  // tap to both. Taps: one s_load_dwordx16 per block of 16.
  {
    constexpr int R = 8, KA = 128;
    const int o0 = static_cast<int>(a0 - js) + R * t;  // local index of the first output
    f2 acc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = f2{0.0f, 0.0f};
#pragma unroll 1
    for (int kb = 0; kb < KA / 16; ++kb) {
      // output i, tap k = 16 kb + kk uses f[o0 + i - k]: window index m = i + 15 - kk
      const int wbase = o0 - 16 * kb - 15;
      f2 w[R + 15];
#pragma unroll
      for (int m = 0; m < R + 15; ++m) w[m] = P[ppos(wbase + m)];
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const f2 tap = splat2(C.a[16 * kb + kk]);
#pragma unroll
        for (int i = 0; i < R; ++i) acc[i] = fma2(tap, w[i + 15 - kk], acc[i]);
      }
    }
    float* __restrict__ y = a.y + ch * a.y_stride;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const long long j = a0 + R * t + i;
      if (j < a_end) y[j] = acc[i].x;
      if (j + kHalf < a_end) y[j + kHalf] = acc[i].y;
    }
  }
  if (last && t < 128) a.carry_out[ch * kWbfmCarry + 8 + t] = get_f(P, static_cast<int>(a.n_dec - 128 + t - js));
}

}  // namespace

int wbfm_front_grid() {
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) ncu = p.multiProcessorCount;
  }
  return ((4 * ncu) + 7) / 8 * 8;  // 4 resident workgroups per CU, a multiple of 8 (XCDs)
}

void launch_wbfm(const WbfmArgs& a, const WbfmFrontConst& f, const WbfmBackConst& b, int nch,
                 hipStream_t s) {
  if (a.n_dec <= 0 || nch <= 0) return;
  static const int G = wbfm_front_grid();
  const bool a16 = (reinterpret_cast<uintptr_t>(a.x) % 16 == 0) && (a.x_stride % 2 == 0);
  const int tiles = div_up(a.n_dec, kWbfmPhi);
  const long long total = static_cast<long long>(tiles) * nch;
  int grid = G;
  if (total < grid) grid = static_cast<int>((total + 7) / 8 * 8);
  if (a16) k_wbfm_front<true><<<grid, NT, 0, s>>>(a, f, tiles, nch);
  else k_wbfm_front<false><<<grid, NT, 0, s>>>(a, f, tiles, nch);
  const dim3 gb(div_up(a.n_dec, kBackA), nch);
  k_wbfm_back<<<gb, NT, 0, s>>>(a, b);
  ORION_LAUNCH_CHECK();
}

}  // namespace orion
