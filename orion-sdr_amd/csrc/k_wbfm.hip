// k_wbfm.hip — the WBFM demodulation chain on gfx950 (the north-star path).
//
// Reference composition (docs/demodulate.md:128-133, SURVEY §3 stack 2):
//   Rotator(-f_off).rotate_block (dsp/rotator.rs:74-85)
//   -> FirDecimator(fs, 8, ...)  (dsp/decim.rs:44-76; kept outputs only here)
//   -> FmQuadratureDemod         (demodulate/fm.rs:45-77: discriminator + LpCascade)
//   -> FirLowpass                (dsp/fir.rs:47-66, the audio filter).
//
// k_wbfm_front — one workgroup (256 lanes) per tile of 512 decimated outputs:
//   stage 4224 cf32 inputs (16-B loads, NCO-mixed with a per-position phasor
//   table) into the polyphase LDS image; polyphase FIR at the kept outputs (two
//   per lane, packed FMA, taps from SGPRs); the tile's common phasor factor is
//   applied to the 512 decimated outputs; the discriminator (atan2_approx op for
//   op) produces 511 phi values (tiles overlap by one decimated sample). No
//   cross-workgroup state: ~16k workgroups per 2^26-sample call, 4 per CU.
// k_wbfm_back — one workgroup per 4096 audio outputs: LpCascade over phi by a
//   state-carry scan (19 samples per lane, f64 Kogge-Stone + cross-wave carry,
//   re-run with the reference's f32 TDF-II update), started 768 samples early
//   from a zero state (pole radius 0.953: the transient is < 1e-8 of the state
//   after 641 samples); then the 125-tap audio FIR.
// The first workgroup of each kernel starts from the exact state carried from
// the previous call (last decimated sample, 128 raw inputs, IIR state, last 128
// IIR outputs), so k calls equal one call on the concatenation.
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

__device__ __forceinline__ float lp4_step(const BiquadK& bq, float (&s)[4], float x) {
  const float y0 = bq.step(s[0], s[1], x);
  return bq.step(s[2], s[3], y0);
}

// Consecutive logical tiles on one XCD (blocks b, b+8, ... share an XCD under the
// observed round-robin dispatch): neighbours' 120-sample halo overlap then hits
// the same L2. Speed only — correctness never depends on placement.
__device__ __forceinline__ int xcd_tile(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return x * q + (x < r ? x : r) + i;
}

template <bool A16>
__global__ __launch_bounds__(NT) void k_wbfm_front(const WbfmArgs a, const WbfmFrontConst C) {
  __shared__ __attribute__((aligned(16))) f2 U[PW::LDS_F2];
  __shared__ __attribute__((aligned(16))) f2 D[T];
  const int t = threadIdx.x;
  const int ch = blockIdx.y;
  const int b = xcd_tile(blockIdx.x, gridDim.x);
  const long long n = a.n;
  const long long J = static_cast<long long>(b) * kWbfmPhi;  // first phi of this tile
  const long long Jd = J - 1;                                 // first decimated output
  const long long porg = static_cast<long long>(M) * (Jd - Q);
  const f2* __restrict__ x = a.x + ch * a.x_stride;
  const f2* __restrict__ hist = a.hist_in + ch * kWbfmHist;
  const f2* __restrict__ tab = a.tab + static_cast<long long>(ch) * PW::NS;

  // ---- stage: 16-B loads, NCO mix, polyphase scatter ----
  f2 v[KP][2];
  if (porg >= 0 && porg + PW::NS <= n) {
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const int p = 2 * t + 2 * NT * k;
      if (p < PW::NS) {
        if constexpr (A16) {
          const f4 w = *reinterpret_cast<const f4*>(x + porg + p);
          v[k][0] = f2{w.x, w.y};
          v[k][1] = f2{w.z, w.w};
        } else {
          v[k][0] = x[porg + p];
          v[k][1] = x[porg + p + 1];
        }
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const int p = 2 * t + 2 * NT * k;
      if (p < PW::NS) {
        v[k][0] = load_hist(x, n, hist, kWbfmHist, porg + p);
        v[k][1] = load_hist(x, n, hist, kWbfmHist, porg + p + 1);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const int p = 2 * t + 2 * NT * k;
    if (p < PW::NS) {
      const f4 tv = *reinterpret_cast<const f4*>(tab + p);  // e^{j theta p}, e^{j theta (p+1)}
      U[PW::slot(p)] = cmul_rot(v[k][0], f2{tv.x, tv.y});
      U[PW::slot(p + 1)] = cmul_rot(v[k][1], f2{tv.z, tv.w});
    }
  }
  __syncthreads();

  // ---- polyphase FIR at the kept outputs; common phasor of the tile ----
  {
    f2 acc[PW::R];
    PW::compute(U, t, [&](int c, int q) { return C.g[c * Q + q]; }, acc);
    const f2 S = phasor_q64(static_cast<uint64_t>(a.k0 + porg + 1), a.step[ch]);
    D[2 * t] = cmul(acc[0], S);
    D[2 * t + 1] = cmul(acc[1], S);
    if (b == 0 && t == 0) {  // d[-1]: the last decimated sample of the previous call
      const float* ci = a.carry_in + ch * kWbfmCarry;
      D[0] = f2{ci[4], ci[5]};
    }
  }
  __syncthreads();

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
    if (t < kWbfmHist) a.hist_out[ch * kWbfmHist + t] = load_hist(x, n, hist, kWbfmHist, n - kWbfmHist + t);
  }
}

// Back-kernel LDS slot of local sample l (l = -128 .. kBackSpan-1): one pad slot
// every 8 so the audio FIR's stride-8-per-lane reads are bank-conflict free.
__device__ __forceinline__ int fpos(int l) { return (l + 128) + ((l + 128) >> 3); }

__global__ __launch_bounds__(NT) void k_wbfm_back(const WbfmArgs a, const WbfmBackConst C) {
  constexpr int H = 128;  // f history slots in front of the span
  __shared__ __attribute__((aligned(16))) float F[((H + kBackSpan + 32) * 9) / 8];
  __shared__ double tot[4][4];
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

  for (int i = t; i < cnt; i += NT) F[fpos(i)] = phi[js + i];
  if (first && t < H) F[fpos(t - H)] = ci[8 + t];  // f[-128 .. -1] from the previous call
  __syncthreads();

  // ---- LpCascade: lane chunk [19 t, 19 t + 19) ----
  float xs[kBackC];
#pragma unroll
  for (int i = 0; i < kBackC; ++i) xs[i] = F[fpos(kBackC * t + i)];
  float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int i = 0; i < kBackC; ++i)
    if (kBackC * t + i < cnt) (void)lp4_step(bq, s, xs[i]);
  double q[4] = {s[0], s[1], s[2], s[3]};
  wave_scan_inclusive<4>(q, C.pw, lane);
  if (lane == 63)
#pragma unroll
    for (int i = 0; i < 4; ++i) tot[wave][i] = q[i];
  __syncthreads();
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
#pragma unroll
  for (int i = 0; i < kBackC; ++i) {
    const int li = kBackC * t + i;
    if (li < cnt) F[fpos(li)] = lp4_step(bq, ef, xs[i]);
  }
  const bool last = a_end == a.n_dec;
  if (last && kBackC * t <= cnt - 1 && cnt - 1 < kBackC * t + kBackC) {
    float* co = a.carry_out + ch * kWbfmCarry;
#pragma unroll
    for (int i = 0; i < 4; ++i) co[i] = ef[i];
  }
  __syncthreads();

  // ---- audio FIR (fir.rs:57-66, quirk-mapped taps) over [a0, a_end) ----
  // Lane t owns outputs a0 + 8t + i and a0 + 2048 + 8t + i (i < 8), accumulated as
  // float2 pairs so one v_pk_fma_f32 applies a tap to both halves; the window
  // pairs (f[j-k], f[j+2048-k]) come from two b32 LDS reads at stride 9 floats per
  // lane (F is padded one slot every 8: conflict-free). Taps: one s_load_dwordx16
  // per block of 16.
  {
    constexpr int R = 8, HALF = kBackA / 2, KA = 128;
    const int o0 = static_cast<int>(a0 - js) + R * t;  // local index of the first output
    f2 acc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = f2{0.0f, 0.0f};
#pragma unroll 1
    for (int kb = 0; kb < KA / 16; ++kb) {
      // output i, tap k = 16 kb + kk uses f[o0 + i - k]: window w = i + 15 - kk
      const int wbase = o0 - 16 * kb - 15;
      f2 w[R + 15];
#pragma unroll
      for (int m = 0; m < R + 15; ++m) w[m] = f2{F[fpos(wbase + m)], F[fpos(wbase + m + HALF)]};
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
      if (j + HALF < a_end) y[j + HALF] = acc[i].y;
    }
  }
  if (last && t < H) a.carry_out[ch * kWbfmCarry + 8 + t] = F[fpos(static_cast<int>(a.n_dec - H + t - js))];
}

}  // namespace

void launch_wbfm(const WbfmArgs& a, const WbfmFrontConst& f, const WbfmBackConst& b, int nch,
                 hipStream_t s) {
  if (a.n_dec <= 0 || nch <= 0) return;
  const bool a16 = (reinterpret_cast<uintptr_t>(a.x) % 16 == 0) && (a.x_stride % 2 == 0);
  const dim3 gf(div_up(a.n_dec, kWbfmPhi), nch);
  if (a16) k_wbfm_front<true><<<gf, NT, 0, s>>>(a, f);
  else k_wbfm_front<false><<<gf, NT, 0, s>>>(a, f);
  const dim3 gb(div_up(a.n_dec, kBackA), nch);
  k_wbfm_back<<<gb, NT, 0, s>>>(a, b);
  ORION_LAUNCH_CHECK();
}

}  // namespace orion
