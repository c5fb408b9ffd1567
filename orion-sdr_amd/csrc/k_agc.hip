// k_agc.hip — AgcRms / AgcRmsIq (dsp/agc.rs:7-150) on the device.
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

namespace orion {
namespace {

struct AgcK {
  float att, rel, tgt, gmin, gmax;
};

template <bool IQ>
__device__ __forceinline__ float agc_x2(const float* in, long long i) {
  if constexpr (IQ) {
    const float2 v = reinterpret_cast<const float2*>(in)[i];
    return v.x * v.x + v.y * v.y;
  } else {
    const float v = in[i];
    return v * v;
  }
}

template <bool IQ>
struct AgcSample {
  using T = typename std::conditional<IQ, float2, float>::type;
};

constexpr int kB = 16;

// Walks samples [s, e) of one lane in batches of kB, the next batch's loads issued
// before the current batch's recurrence. OUT = false: envelope only (the warm-up).
template <bool IQ, bool OUT>
__device__ __forceinline__ float agc_walk(const typename AgcSample<IQ>::T* __restrict__ x,
                                          typename AgcSample<IQ>::T* __restrict__ y, long long s, long long e,
                                          float env, const AgcK& k, float oma, float omr) {
  using T = typename AgcSample<IQ>::T;
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
      float re, im = 0.0f, x2;
      if constexpr (IQ) {
        re = cur[j].x; im = cur[j].y;
        x2 = re * re + im * im;
      } else {
        re = cur[j];
        x2 = re * re;
      }
      const bool up = x2 > env;
      const float a = up ? k.att : k.rel;
      const float om = up ? oma : omr;
      const float ne = a * env + om * x2;  // agc.rs:40
      if (i < e) {
        env = ne;
        if constexpr (OUT) {
          const float rms = fmaxf(sqrtf(env), 1e-6f);
          const float g = fminf(fmaxf(k.tgt / rms, k.gmin), k.gmax);
          if constexpr (IQ) {
            y[i] = make_float2(g * re, g * im);
          } else {
            y[i] = g * re;
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) cur[j] = nxt[j];
  }
  return env;
}

// One wave walks samples [s, e) in order from env (the re-runs of k_agc_fix and the
// sequential path). The 64 lanes load 64 samples and form x2 and both candidate
// (1 - a) * x2 products; the envelope chain itself is uniform across the wave
// (x2 and the products read lane by lane into SGPRs: compare, two selects, one
// multiply, one add per sample), then every lane forms its sample's gain and
// output. Same f32 ops and roundings as agc.rs:40 and :63-67.
template <bool IQ>
__device__ __forceinline__ float agc_wave_walk(const typename AgcSample<IQ>::T* __restrict__ x,
                                               typename AgcSample<IQ>::T* __restrict__ y, long long s, long long e,
                                               float env, const AgcK& k, float oma, float omr) {
  using T = typename AgcSample<IQ>::T;
  const int lane = threadIdx.x & 63;
  T cur = s + lane < e ? x[s + lane] : T{};
  for (long long base = s; base < e; base += 64) {
    const long long i = base + lane;
    const T nxt = i + 64 < e ? x[i + 64] : T{};
    float re, im = 0.0f, x2;
    if constexpr (IQ) {
      re = cur.x; im = cur.y;
      x2 = re * re + im * im;
    } else {
      re = cur;
      x2 = re * re;
    }
    const float pa = oma * x2, pr = omr * x2;
    const int cnt = e - base < 64 ? static_cast<int>(e - base) : 64;
    float mine = 0.0f;
    if (cnt == 64) {
#pragma unroll
      for (int j = 0; j < 64; ++j) {
        const float xj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x2), j));
        const float aj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pa), j));
        const float rj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pr), j));
        const bool up = xj > env;
        env = (up ? k.att : k.rel) * env + (up ? aj : rj);
        mine = lane == j ? env : mine;
      }
    } else {
      for (int j = 0; j < cnt; ++j) {
        const float xj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x2), j));
        const float aj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pa), j));
        const float rj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pr), j));
        const bool up = xj > env;
        env = (up ? k.att : k.rel) * env + (up ? aj : rj);
        mine = lane == j ? env : mine;
      }
    }
    if (i < e) {
      const float rms = fmaxf(sqrtf(mine), 1e-6f);
      const float g = fminf(fmaxf(k.tgt / rms, k.gmin), k.gmax);
      if constexpr (IQ) {
        y[i] = make_float2(g * re, g * im);
      } else {
        y[i] = g * re;
      }
    }
    cur = nxt;
  }
  return env;
}

// The whole call in order by one wave (warm-ups as long as the call itself).
template <bool IQ>
__global__ __launch_bounds__(64) void k_agc_seq(const float* __restrict__ in, float* __restrict__ out, long long n,
                                                AgcK k, const float* __restrict__ env_in,
                                                float* __restrict__ env_out) {
  using T = typename AgcSample<IQ>::T;
  float env = env_in[0];
  if (env == 0.0f) env = fmaxf(agc_x2<IQ>(in, 0), 1e-12f);  // agc.rs:57-60
  const float oma = 1.0f - k.att, omr = 1.0f - k.rel;
  env = agc_wave_walk<IQ>(reinterpret_cast<const T*>(in), reinterpret_cast<T*>(out), 0, n, env, k, oma, omr);
  if (threadIdx.x == 0) env_out[0] = env;
}

// Pass 1: chunk c = [c*L, min(c*L+L, n)), warm-up from max(c*L - W, 0).
template <bool IQ>
__global__ __launch_bounds__(256) void k_agc(const float* __restrict__ in, float* __restrict__ out,
                                             long long n, long long L, long long W, AgcK k,
                                             const float* __restrict__ env_in, float* __restrict__ env_out,
                                             float* __restrict__ ent, float* __restrict__ ext,
                                             long long* __restrict__ first_bad) {
  using T = typename AgcSample<IQ>::T;
  const T* x = reinterpret_cast<const T*>(in);
  T* y = reinterpret_cast<T*>(out);
  const long long c = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const long long b = c * L;
  if (b >= n) return;
  if (c == 0) first_bad[0] = (n + L - 1) / L;  // "no disagreement" until k_agc_check says otherwise
  const long long e = b + L < n ? b + L : n;
  // A warm-up that would reach back past the call's first sample starts there, from
  // the carried envelope, exactly as chunk 0 does (such chunks are exact).
  const long long s0 = b - W > 0 ? b - W : 0;
  float env;
  if (s0 == 0) {
    env = env_in[0];
    if (env == 0.0f) env = fmaxf(agc_x2<IQ>(in, 0), 1e-12f);  // agc.rs:57-60
  } else {
    env = fmaxf(agc_x2<IQ>(in, s0), 1e-12f);
  }
  const float oma = 1.0f - k.att, omr = 1.0f - k.rel;  // (1 - a) as agc.rs:40 forms it
  env = agc_walk<IQ, false>(x, y, s0, b, env, k, oma, omr);
  ent[c] = env;
  env = agc_walk<IQ, true>(x, y, b, e, env, k, oma, omr);
  ext[c] = env;
  if (e == n) env_out[0] = env;
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
template <bool IQ>
__global__ __launch_bounds__(64) void k_agc_fix(const float* __restrict__ in, float* __restrict__ out,
                                                long long n, long long L, AgcK k, const float* __restrict__ ent,
                                                const float* __restrict__ ext, const long long* __restrict__ first_bad,
                                                float* __restrict__ env_out) {
  using T = typename AgcSample<IQ>::T;
  const T* x = reinterpret_cast<const T*>(in);
  T* y = reinterpret_cast<T*>(out);
  const long long chunks = (n + L - 1) / L;
  long long c = first_bad[0];
  if (c >= chunks) return;
  const int lane = threadIdx.x;
  const float oma = 1.0f - k.att, omr = 1.0f - k.rel;
  float ex = ext[c - 1];  // chunks < c are consistent, so this exit is the sequential one
  while (c < chunks) {
    // chunk c entered with the wrong envelope: re-run it from ex, in order
    const long long b = c * L, e = b + L < n ? b + L : n;
    ex = agc_wave_walk<IQ>(x, y, b, e, ex, k, oma, omr);
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

class AgcBlock final : public Block {
 public:
  AgcBlock(bool iq, float fs, float attack_ms, float release_ms, float target_rms) : iq_(iq) {
    // agc.rs:21 / :97: a(ms) = exp(-1 / (fs * (max(ms, 1e-3) / 1000)))
    auto coef = [fs](float ms) { return std::exp(-1.0f / (fs * (std::max(ms, 1e-3f) / 1000.0f))); };
    k_.att = coef(attack_ms);
    k_.rel = coef(release_ms);
    k_.tgt = std::max(target_rms, 1e-6f);
    k_.gmin = 0.05f;
    k_.gmax = 20.0f;
    const double amax = std::max(k_.att, k_.rel);
    // amax^W < 1e-9; amax == 1 (or NaN) never forgets: one sequential lane.
    warm_ = amax < 1.0 ? static_cast<long long>(std::ceil(std::log(1e-9) / std::log(amax))) : -1;
    if (const char* v = std::getenv("ORION_AGC_WORK_DIV")) work_div_ = std::max(1LL, std::atoll(v));
    if (const char* v = std::getenv("ORION_AGC_MIN_L")) min_l_ = std::max(1LL, std::atoll(v));
    if (const char* v = std::getenv("ORION_AGC_SEQ_DIV")) seq_div_ = std::max(1LL, std::atoll(v));
    env_.resize(2 * sizeof(float));
    env_.zero();
  }
  const char* name() const override { return iq_ ? "AgcRmsIq" : "AgcRms"; }
  Dt in_type() const override { return iq_ ? Dt::C32 : Dt::F32; }
  Dt out_type() const override { return iq_ ? Dt::C32 : Dt::F32; }
  bool alias_ok() const override { return true; }  // overlapping in/out: staged through a copy
  // Chunk length: the extra warm-up work per chunk is W/L of a chunk, so L >= W/div
  // caps the total work at (1 + div) x n; the floor keeps >> 1024 waves busy for
  // short warm-ups. W >= n/4: one wave walks the call in order (k_agc_seq, ~27 ns
  // per sample, faster than lanes whose own walks are that long).
  long long chunk_len(long long n) const {
    if (warm_ < 0 || warm_ >= n / seq_div_) return n;
    return std::max(min_l_, (warm_ + work_div_ - 1) / work_div_);
  }
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
    const long long L = chunk_len(n);
    const long long chunks = (n + L - 1) / L;
    float* e = env_.as<float>();
    float* ein = e + cur_;
    float* eout = e + (cur_ ^ 1);
    if (chunks == 1) {  // one wave, in order
      if (iq_) {
        hipLaunchKernelGGL(k_agc_seq<true>, dim3(1), dim3(64), 0, s, static_cast<const float*>(in),
                           static_cast<float*>(out), n, k_, ein, eout);
      } else {
        hipLaunchKernelGGL(k_agc_seq<false>, dim3(1), dim3(64), 0, s, static_cast<const float*>(in),
                           static_cast<float*>(out), n, k_, ein, eout);
      }
      ORION_HIP(hipGetLastError());
      cur_ ^= 1;
      return {static_cast<size_t>(n), static_cast<size_t>(n)};
    }
    const size_t need = static_cast<size_t>(chunks) * 2 * sizeof(float) + sizeof(long long);
    if (chunk_state_.size() < need) chunk_state_.resize(need);
    long long* first_bad = chunk_state_.as<long long>();
    float* ent = reinterpret_cast<float*>(first_bad + 1);
    float* ext = ent + chunks;
    const unsigned grid = static_cast<unsigned>((chunks + 255) / 256);
    const long long W = warm_ < 0 ? 0 : warm_;
    const float* x = static_cast<const float*>(in);
    float* y = static_cast<float*>(out);
    if (iq_) {
      hipLaunchKernelGGL(k_agc<true>, dim3(grid), dim3(256), 0, s, x, y, n, L, W, k_, ein, eout, ent, ext, first_bad);
    } else {
      hipLaunchKernelGGL(k_agc<false>, dim3(grid), dim3(256), 0, s, x, y, n, L, W, k_, ein, eout, ent, ext, first_bad);
    }
    ORION_HIP(hipGetLastError());
    {
      hipLaunchKernelGGL(k_agc_check, dim3(static_cast<unsigned>((chunks - 1 + 255) / 256)), dim3(256), 0, s, ent,
                         ext, chunks, first_bad);
      ORION_HIP(hipGetLastError());
      if (iq_) {
        hipLaunchKernelGGL(k_agc_fix<true>, dim3(1), dim3(64), 0, s, x, y, n, L, k_, ent, ext, first_bad, eout);
      } else {
        hipLaunchKernelGGL(k_agc_fix<false>, dim3(1), dim3(64), 0, s, x, y, n, L, k_, ent, ext, first_bad, eout);
      }
      ORION_HIP(hipGetLastError());
    }
    cur_ ^= 1;
    return {static_cast<size_t>(n), static_cast<size_t>(n)};
  }
  void reset() override {
    env_.zero();
    cur_ = 0;
  }
  std::vector<float> taps(int which) const override {
    if (which == 1) return {static_cast<float>(chunk_len(1LL << 24))};
    return {k_.att, k_.rel, k_.tgt, static_cast<float>(warm_)};
  }

 private:
  bool iq_;
  AgcK k_{};
  long long warm_ = 0;
  long long work_div_ = 16, min_l_ = 256, seq_div_ = 4;
  DevBuf env_;          // two floats: the carried envelope, ping-ponged per call
  DevBuf chunk_state_;  // first disagreeing chunk, then ent[chunks], ext[chunks]
  DevBuf copy_;         // input copy for overlapping in/out
  int cur_ = 0;
};

}  // namespace

std::unique_ptr<Block> make_agc(bool iq, float fs, float attack_ms, float release_ms, float target_rms) {
  return std::make_unique<AgcBlock>(iq, fs, attack_ms, release_ms, target_rms);
}

}  // namespace orion
