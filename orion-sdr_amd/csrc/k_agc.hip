// k_agc.hip — AgcRms / AgcRmsIq (dsp/agc.rs:7-150) and CwKeyedMod (modulate/cw.rs:9-87)
// on the device: both are the same switched one-pole envelope recurrence.
//
// The reference's envelope is a data-dependent recurrence
//   env <- a(x2 > env) * env + (1 - a) * x2,  a in {attack_a, release_a}
// (agc.rs:33-41). In real arithmetic it is a continuous piecewise-linear map of
// env with slopes <= amax = max(attack_a, release_a), so two trajectories over the
// same input approach each other by amax per sample. Pass 1 (k_agc) exploits
// that: each lane owns a chunk of L samples, starts W samples early (amax^W <
// 1e-9, an envelope-only walk) from the reference's seed rule applied there, and
// records the envelope it entered its chunk with (ent[c]) and the one it left
// with (ext[c]).
//
// In f32 the contraction is NOT guaranteed: near a constant x2 with a close to 1
// the rounded map has a band of exact fixed points about ulp/(1-a) wide, and a
// warm-up trajectory can settle on a different fixed point than the sequential
// one. So exactness is proved, not assumed: chunk c's outputs are the sequential
// ones iff its entering envelope equals chunk c-1's true exit (by induction from
// chunk 0, which starts from the carried state). k_agc_check finds the first
// chunk whose ent differs (bitwise) from its predecessor's ext; k_agc_fix (one
// wave) re-runs from there, one chunk after another from the true exit, until a
// chunk's recorded entry agrees again, then searches for the next disagreement.
// Every output is therefore the reference's sequential f32 result. Typical
// signals need no re-run; a long constant stretch (the ADVICE case) degrades to an
// in-order walk of the stretch (agc_wave_walk, ~27 ns per sample), never to a
// wrong answer.
//
// Per sample: the reference's f32 ops in its order, no FMA contraction
// (-ffp-contract=off), correctly rounded sqrt and divide.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "blocks.hpp"
#include "hip_common.hpp"
#include "osc.hpp"

namespace orion {
namespace {

struct AgcK {
  float att, rel, tgt, gmin, gmax;
};

// The switched one-pole envelope, env <- a * env + (1 - a) * d with a = att when
// up(d, env) else rel, as a policy over the per-sample ops (the walks and the
// exactness machinery below are shared):
//   AgcPol<IQ> — dsp/agc.rs:33-75 / :124-150: d = |x|^2, up = d > env, seed env = max(d0,
//     1e-12) when the carried env is 0 (agc.rs:57-60), out = clamp(tgt / max(sqrt(env),
//     1e-6), gmin, gmax) * x.
//   CwPol — modulate/cw.rs:45-87 CwKeyedMod: d = clamp(x, 0, 1), up = d >= env, no
//     reseed, out = mix_with_nco((env * gain, 0), nco) (the non-FMA product, nco.rs:63-66)
//     with the tone Nco's phasor (osc.hpp RefOsc: the reference recurrence, tabulated).
template <bool IQ>
struct AgcPol {
  using In = typename std::conditional<IQ, float2, float>::type;
  using Out = In;
  AgcK k;
  float att, rel, oma, omr;
  __device__ __forceinline__ float drive(In v) const {
    if constexpr (IQ) return v.x * v.x + v.y * v.y;
    else return v * v;
  }
  __device__ __forceinline__ bool up(float d, float env) const { return d > env; }
  __device__ __forceinline__ float seed(float env, float d0) const { return env == 0.0f ? fmaxf(d0, 1e-12f) : env; }
  __device__ __forceinline__ float warm_seed(float d) const { return fmaxf(d, 1e-12f); }
  __device__ __forceinline__ Out out(In v, float env, long long) const {
    const float rms = fmaxf(sqrtf(env), 1e-6f);
    const float g = fminf(fmaxf(k.tgt / rms, k.gmin), k.gmax);
    if constexpr (IQ) return make_float2(g * v.x, g * v.y);
    else return g * v;
  }
};
struct CwPol {
  using In = float;
  using Out = float2;
  float att, rel, oma, omr, gain;
  uint64_t k0;  // sample i of the call: oscillator output k0 + i (the Nco, cw.rs:27)
  OscDev osc;
  __device__ __forceinline__ float drive(In v) const { return v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v); }  // f32::clamp
  __device__ __forceinline__ bool up(float d, float env) const { return d >= env; }
  __device__ __forceinline__ float seed(float env, float) const { return env; }
  __device__ __forceinline__ float warm_seed(float d) const { return d; }
  __device__ __forceinline__ Out out(In, float env, long long i) const {
    const float m = env * gain;
    const f2 p = osc_at(osc, k0 + static_cast<uint64_t>(i));
    return make_float2(m * p.x - 0.0f * p.y, m * p.y + 0.0f * p.x);
  }
};

constexpr int kB = 16;

// Walks samples [s, e) of one lane in batches of kB, the next batch's loads issued
// before the current batch's recurrence. OUT = false: envelope only (the warm-up).
template <class Pol, bool OUT>
__device__ __forceinline__ float agc_walk(const typename Pol::In* __restrict__ x, typename Pol::Out* __restrict__ y,
                                          long long s, long long e, float env, const Pol& P) {
  using T = typename Pol::In;
  T cur[kB], nxt[kB];
#pragma unroll
  for (int j = 0; j < kB; ++j) cur[j] = s + j < e ? x[s + j] : T{};
  for (long long base = s; base < e; base += kB) {
    const long long nb = base + kB;
#pragma unroll
    for (int j = 0; j < kB; ++j) nxt[j] = nb + j < e ? x[nb + j] : T{};
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      const long long i = base + j;
      const float d = P.drive(cur[j]);
      const bool up = P.up(d, env);
      const float ne = (up ? P.att : P.rel) * env + (up ? P.oma : P.omr) * d;  // agc.rs:40, cw.rs:58-62
      if (i < e) {
        env = ne;
        if constexpr (OUT) y[i] = P.out(cur[j], env, i);
      }
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) cur[j] = nxt[j];
  }
  return env;
}

// One wave walks samples [s, e) in order from env (the re-runs of k_agc_fix, the
// sequential path and the long-warm-up chunks of k_agc_wave). The 64 lanes load 64
// samples and form d and both candidate (1 - a) * d products; the envelope chain
// itself is uniform across the wave (d and the products read lane by lane: compare,
// two selects, one multiply, one add per sample), then every lane forms its
// sample's output. Same f32 ops and roundings as the reference's per-sample
// update. OUT = false: envelope only (a warm-up).
template <class Pol, bool OUT = true>
__device__ __forceinline__ float agc_wave_walk(const typename Pol::In* __restrict__ x,
                                               typename Pol::Out* __restrict__ y, long long s, long long e, float env,
                                               const Pol& P) {
  using T = typename Pol::In;
  const int lane = threadIdx.x & 63;
  T cur = s + lane < e ? x[s + lane] : T{};
  for (long long base = s; base < e; base += 64) {
    const long long i = base + lane;
    const T nxt = i + 64 < e ? x[i + 64] : T{};
    const float d = P.drive(cur);
    const float pa = P.oma * d, pr = P.omr * d;
    const int cnt = e - base < 64 ? static_cast<int>(e - base) : 64;
    float mine = 0.0f;
    if (cnt == 64) {
#pragma unroll
      for (int j = 0; j < 64; ++j) {
        const float xj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d), j));
        const float aj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pa), j));
        const float rj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pr), j));
        const bool up = P.up(xj, env);
        env = (up ? P.att : P.rel) * env + (up ? aj : rj);
        if constexpr (OUT) mine = lane == j ? env : mine;
      }
    } else {
      for (int j = 0; j < cnt; ++j) {
        const float xj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d), j));
        const float aj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pa), j));
        const float rj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pr), j));
        const bool up = P.up(xj, env);
        env = (up ? P.att : P.rel) * env + (up ? aj : rj);
        if constexpr (OUT) mine = lane == j ? env : mine;
      }
    }
    if constexpr (OUT) {
      if (i < e) y[i] = P.out(cur, mine, i);
    }
    cur = nxt;
  }
  return env;
}

// The whole call in order by one wave (warm-ups as long as the call itself).
template <class Pol>
__global__ __launch_bounds__(64) void k_agc_seq(const void* __restrict__ in, void* __restrict__ out, long long n,
                                                Pol P, const float* __restrict__ env_in, float* __restrict__ env_out) {
  const auto* x = static_cast<const typename Pol::In*>(in);
  float env = P.seed(env_in[0], P.drive(x[0]));
  env = agc_wave_walk<Pol>(x, static_cast<typename Pol::Out*>(out), 0, n, env, P);
  if (threadIdx.x == 0) env_out[0] = env;
}

// Pass 1: chunk c = [c*L, min(c*L+L, n)), warm-up from max(c*L - W, 0).
template <class Pol>
__global__ __launch_bounds__(256) void k_agc(const void* __restrict__ in, void* __restrict__ out, long long n,
                                             long long L, long long W, Pol P, const float* __restrict__ env_in,
                                             float* __restrict__ env_out, float* __restrict__ ent,
                                             float* __restrict__ ext, long long* __restrict__ first_bad) {
  const auto* x = static_cast<const typename Pol::In*>(in);
  auto* y = static_cast<typename Pol::Out*>(out);
  const long long c = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const long long b = c * L;
  if (b >= n) return;
  if (c == 0) first_bad[0] = (n + L - 1) / L;  // "no disagreement" until k_agc_check says otherwise
  const long long e = b + L < n ? b + L : n;
  // A warm-up that would reach back past the call's first sample starts there, from
  // the carried envelope, exactly as chunk 0 does (such chunks are exact).
  const long long s0 = b - W > 0 ? b - W : 0;
  float env = s0 == 0 ? P.seed(env_in[0], P.drive(x[0])) : P.warm_seed(P.drive(x[s0]));
  env = agc_walk<Pol, false>(x, y, s0, b, env, P);
  ent[c] = env;
  env = agc_walk<Pol, true>(x, y, b, e, env, P);
  ext[c] = env;
  if (e == n) env_out[0] = env;
}

// Pass 1 for long warm-ups (few chunks: a lane per chunk would leave the chip
// idle and walk W samples with its own strided loads, ~110 ns per sample): one
// wave per chunk, warm-up and chunk by the wave walk (coalesced, ~27 ns per
// sample). Same ent / ext records as k_agc.
template <class Pol>
__global__ __launch_bounds__(64) void k_agc_wave(const void* __restrict__ in, void* __restrict__ out, long long n,
                                                 long long L, long long W, Pol P, const float* __restrict__ env_in,
                                                 float* __restrict__ env_out, float* __restrict__ ent,
                                                 float* __restrict__ ext, long long* __restrict__ first_bad) {
  const auto* x = static_cast<const typename Pol::In*>(in);
  auto* y = static_cast<typename Pol::Out*>(out);
  const long long c = blockIdx.x;
  const long long b = c * L;
  const bool lead = threadIdx.x == 0;
  if (c == 0 && lead) first_bad[0] = (n + L - 1) / L;
  const long long e = b + L < n ? b + L : n;
  const long long s0 = b - W > 0 ? b - W : 0;
  float env = s0 == 0 ? P.seed(env_in[0], P.drive(x[0])) : P.warm_seed(P.drive(x[s0]));
  env = agc_wave_walk<Pol, false>(x, y, s0, b, env, P);
  if (lead) ent[c] = env;
  env = agc_wave_walk<Pol, true>(x, y, b, e, env, P);
  if (lead) {
    ext[c] = env;
    if (e == n) env_out[0] = env;
  }
}

// Pass 2: the first chunk whose entering envelope is not (bitwise) its
// predecessor's exit.
__global__ __launch_bounds__(256) void k_agc_check(const float* __restrict__ ent, const float* __restrict__ ext,
                                                   long long chunks, long long* __restrict__ first_bad) {
  const long long c = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x + 1;
  if (c >= chunks) return;
  if (__float_as_uint(ent[c]) != __float_as_uint(ext[c - 1]))
    atomicMin(reinterpret_cast<unsigned long long*>(first_bad), static_cast<unsigned long long>(c));
}

// Pass 3 (one wave): re-run disagreeing chunks in order from the true exit of
// their predecessor. Exits immediately when pass 2 found nothing.
template <class Pol>
__global__ __launch_bounds__(64) void k_agc_fix(const void* __restrict__ in, void* __restrict__ out, long long n,
                                                long long L, Pol P, const float* __restrict__ ent,
                                                const float* __restrict__ ext, const long long* __restrict__ first_bad,
                                                float* __restrict__ env_out) {
  const auto* x = static_cast<const typename Pol::In*>(in);
  auto* y = static_cast<typename Pol::Out*>(out);
  const long long chunks = (n + L - 1) / L;
  long long c = first_bad[0];
  if (c >= chunks) return;
  const int lane = threadIdx.x;
  float ex = ext[c - 1];  // chunks < c are consistent, so this exit is the sequential one
  while (c < chunks) {
    // chunk c entered with the wrong envelope: re-run it from ex, in order
    const long long b = c * L, e = b + L < n ? b + L : n;
    ex = agc_wave_walk<Pol>(x, y, b, e, ex, P);
    ++c;
    // the next chunk whose recorded entry is not the true exit of its predecessor
    long long nxt = chunks;
    for (long long base = c; base < chunks; base += 64) {
      const long long i = base + lane;
      bool bad = false;
      if (i < chunks) {
        const float pred = i == c ? ex : ext[i - 1];
        bad = __float_as_uint(ent[i]) != __float_as_uint(pred);
      }
      const unsigned long long m = __ballot(bad);
      if (m) {
        nxt = base + __ffsll(static_cast<long long>(m)) - 1;
        break;
      }
    }
    if (nxt >= chunks) {
      if (lane == 0) env_out[0] = c == chunks ? ex : ext[chunks - 1];
      return;
    }
    if (nxt != c) ex = ext[nxt - 1];
    c = nxt;
  }
  if (lane == 0) env_out[0] = ex;
}

// Host driver of the three passes for one policy. Chunk length: the extra warm-up
// work per chunk is W/L of a chunk, so L >= W/16 caps the total work at 17 x n; the
// floor keeps >> 1024 waves busy for short warm-ups. W >= n/4: one wave walks the
// call in order (k_agc_seq, ~27 ns per sample, faster than lanes whose own walks are
// that long).
class EnvelopeRunner {
 public:
  explicit EnvelopeRunner(double amax) {
    // amax^W < 1e-9; amax == 1 (or NaN) never forgets: one sequential lane.
    warm_ = amax < 1.0 ? static_cast<long long>(std::ceil(std::log(1e-9) / std::log(amax))) : -1;
    env_.resize(2 * sizeof(float));
    env_.zero();
  }
  long long warm() const { return warm_; }
  long long chunk_len(long long n) const {
    if (warm_ < 0 || warm_ >= n / 4) return n;
    return std::max(256LL, (warm_ + 15) / 16);
  }
  template <class Pol>
  void run(const void* in, void* out, long long n, const Pol& P, hipStream_t s) {
    const long long L = chunk_len(n);
    const long long chunks = (n + L - 1) / L;
    float* e = env_.as<float>();
    float* ein = e + cur_;
    float* eout = e + (cur_ ^ 1);
    cur_ ^= 1;
    if (chunks == 1) {  // one wave, in order
      hipLaunchKernelGGL(k_agc_seq<Pol>, dim3(1), dim3(64), 0, s, in, out, n, P, ein, eout);
      ORION_HIP(hipGetLastError());
      return;
    }
    const size_t need = static_cast<size_t>(chunks) * 2 * sizeof(float) + sizeof(long long);
    if (chunk_state_.size() < need) chunk_state_.resize(need);
    long long* first_bad = chunk_state_.as<long long>();
    float* ent = reinterpret_cast<float*>(first_bad + 1);
    float* ext = ent + chunks;
    const unsigned grid = static_cast<unsigned>((chunks + 255) / 256);
    const long long W = warm_ < 0 ? 0 : warm_;
    if (chunks <= kWaveChunks) {
      hipLaunchKernelGGL(k_agc_wave<Pol>, dim3(static_cast<unsigned>(chunks)), dim3(64), 0, s, in, out, n, L, W, P, ein,
                         eout, ent, ext, first_bad);
    } else {
      hipLaunchKernelGGL(k_agc<Pol>, dim3(grid), dim3(256), 0, s, in, out, n, L, W, P, ein, eout, ent, ext, first_bad);
    }
    ORION_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_agc_check, dim3(static_cast<unsigned>((chunks - 1 + 255) / 256)), dim3(256), 0, s, ent, ext,
                       chunks, first_bad);
    ORION_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_agc_fix<Pol>, dim3(1), dim3(64), 0, s, in, out, n, L, P, ent, ext, first_bad, eout);
    ORION_HIP(hipGetLastError());
  }
  void reset() {
    env_.zero();
    cur_ = 0;
  }

 private:
  // Up to this many chunks (four waves per SIMD), a wave per chunk (k_agc_wave).
  static constexpr long long kWaveChunks = 4096;
  long long warm_ = 0;
  DevBuf env_;          // two floats: the carried envelope, ping-ponged per call
  DevBuf chunk_state_;  // first disagreeing chunk, then ent[chunks], ext[chunks]
  int cur_ = 0;
};

class AgcBlock final : public Block {
 public:
  AgcBlock(bool iq, float fs, float attack_ms, float release_ms, float target_rms)
      : iq_(iq), runner_(amax_of(fs, attack_ms, release_ms)) {
    // agc.rs:21 / :97: a(ms) = exp(-1 / (fs * (max(ms, 1e-3) / 1000)))
    k_.att = coef(fs, attack_ms);
    k_.rel = coef(fs, release_ms);
    k_.tgt = std::max(target_rms, 1e-6f);
    k_.gmin = 0.05f;
    k_.gmax = 20.0f;
  }
  const char* name() const override { return iq_ ? "AgcRmsIq" : "AgcRms"; }
  Dt in_type() const override { return iq_ ? Dt::C32 : Dt::F32; }
  Dt out_type() const override { return iq_ ? Dt::C32 : Dt::F32; }
  size_t chunk_quantum() const override { return 1; }  // outputs are the sequential recurrence's, bit for bit
  bool alias_ok() const override { return true; }  // overlapping in/out: staged through a copy
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const long long n = static_cast<long long>(std::min(n_in, out_cap));  // agc.rs:49
    if (n == 0) return {0, 0};
    const size_t bytes = static_cast<size_t>(n) * (iq_ ? 8 : 4);
    const char* ib = static_cast<const char*>(in);
    char* ob = static_cast<char*>(out);
    if (ib < ob + bytes && ob < ib + bytes) {
      // the warm-ups and re-runs read inputs other lanes overwrite: work from a copy
      copy_.resize(std::max(copy_.size(), bytes));
      ORION_HIP(hipMemcpyAsync(copy_.as<void>(), in, bytes, hipMemcpyDeviceToDevice, s));
      in = copy_.as<void>();
    }
    const float oma = 1.0f - k_.att, omr = 1.0f - k_.rel;  // (1 - a) as agc.rs:40 forms it
    if (iq_) runner_.run(in, out, n, AgcPol<true>{k_, k_.att, k_.rel, oma, omr}, s);
    else runner_.run(in, out, n, AgcPol<false>{k_, k_.att, k_.rel, oma, omr}, s);
    return {static_cast<size_t>(n), static_cast<size_t>(n)};
  }
  void reset() override { runner_.reset(); }
  std::vector<float> taps(int which) const override {
    if (which == 1) return {static_cast<float>(runner_.chunk_len(1LL << 24))};
    return {k_.att, k_.rel, k_.tgt, static_cast<float>(runner_.warm())};
  }

 private:
  static float coef(float fs, float ms) { return std::exp(-1.0f / (fs * (std::max(ms, 1e-3f) / 1000.0f))); }
  static double amax_of(float fs, float a, float r) { return std::max(coef(fs, a), coef(fs, r)); }
  bool iq_;
  AgcK k_{};
  EnvelopeRunner runner_;
  DevBuf copy_;  // input copy for overlapping in/out
};

// modulate/cw.rs:9-87 CwKeyedMod: keying envelope f32 -> cf32 IQ.
class CwModBlock final : public Block {
 public:
  CwModBlock(float fs, float tone_hz, float rise_ms, float fall_ms)
      : osc_(tone_hz, fs), runner_(std::max(alpha(fs, rise_ms), alpha(fs, fall_ms))) {
    rise_ = alpha(fs, rise_ms);
    fall_ = alpha(fs, fall_ms);
  }
  const char* name() const override { return "CwKeyedMod"; }
  Dt in_type() const override { return Dt::F32; }
  Dt out_type() const override { return Dt::C32; }
  size_t chunk_quantum() const override { return 1; }  // outputs are the sequential recurrence's, bit for bit
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const long long n = static_cast<long long>(std::min(n_in, out_cap));  // cw.rs:47
    if (n == 0) return {0, 0};
    runner_.run(in, out, n, CwPol{rise_, fall_, 1.0f - rise_, 1.0f - fall_, g_, osc_.count(), osc_.dev(n, s)}, s);
    osc_.advance(static_cast<uint64_t>(n));
    return {static_cast<size_t>(n), static_cast<size_t>(n)};
  }
  void reset() override {
    runner_.reset();
    osc_.reset();
  }
  void set_gain(float g) { g_ = g; }  // cw.rs:39-41
  int configure(int option, long long value) override {
    if (option != kOptNcoTable) return -4;
    if (value < 0 || static_cast<unsigned long long>(value) > kNcoTableMax) return -3;
    osc_.set_budget(static_cast<uint64_t>(value));
    return 0;
  }
  std::vector<float> taps(int) const override { return {rise_, fall_, osc_.osc().w_re, osc_.osc().w_im}; }

 private:
  // cw.rs:27-30: tau = (max(ms, 0.1) * 1e-3) * fs; alpha = exp(-1 / tau)
  static float alpha(float fs, float ms) { return std::exp(-1.0f / ((std::max(ms, 0.1f) * 1e-3f) * fs)); }
  RefOsc osc_;
  EnvelopeRunner runner_;
  float rise_ = 0, fall_ = 0, g_ = 1.0f;
};

}  // namespace

std::unique_ptr<Block> make_agc(bool iq, float fs, float attack_ms, float release_ms, float target_rms) {
  return std::make_unique<AgcBlock>(iq, fs, attack_ms, release_ms, target_rms);
}
std::unique_ptr<Block> make_cw_mod(float fs, float tone_hz, float rise_ms, float fall_ms) {
  return std::make_unique<CwModBlock>(fs, tone_hz, rise_ms, fall_ms);
}
int cw_mod_set_gain(Block* b, float g) {
  auto* c = dynamic_cast<CwModBlock*>(b);
  if (!c) return -4;
  c->set_gain(g);
  return 0;
}

}  // namespace orion
