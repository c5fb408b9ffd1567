// k_agc.hip — AgcRms / AgcRmsIq (dsp/agc.rs:7-150) on the device.
//
// The reference's envelope is a data-dependent recurrence
//   env <- a(x2 > env) * env + (1 - a) * x2,  a in {attack_a, release_a}
// (agc.rs:33-41). As a map of env it is continuous at env = x2 (both branches give
// x2) and piecewise linear with slopes attack_a and release_a, so two trajectories
// over the same input approach each other by at least amax = max(attack_a,
// release_a) per sample. Each lane owns a chunk of L samples and starts W samples
// early from a guess (the seed rule of agc.rs:57-60 applied at that sample); the
// host picks W with amax^W < 1e-9, so the entering envelope of every chunk is the
// sequential one to |env error| <= 1e-9 * max x2 (in practice the f32 trajectories
// meet exactly). Chunk 0 starts from the carried state, as the reference does.
// Per sample: the reference's f32 ops in its order, no FMA contraction
// (-ffp-contract=off), correctly rounded sqrt and divide.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
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

template <bool IQ>
__global__ __launch_bounds__(256) void k_agc(const float* __restrict__ in, float* __restrict__ out,
                                             long long n, long long L, long long W, AgcK k,
                                             const float* __restrict__ env_in, float* __restrict__ env_out) {
  using T = typename AgcSample<IQ>::T;
  const T* x = reinterpret_cast<const T*>(in);
  T* y = reinterpret_cast<T*>(out);
  const long long c = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const long long b = c * L;
  if (b >= n) return;
  const long long e = b + L < n ? b + L : n;
  // A warm-up that would reach back past the call's first sample starts there, from
  // the carried envelope, exactly as chunk 0 does.
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
  env = agc_walk<IQ, true>(x, y, b, e, env, k, oma, omr);
  if (e == n) env_out[0] = env;
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
    env_.resize(2 * sizeof(float));
    env_.zero();
  }
  const char* name() const override { return iq_ ? "AgcRmsIq" : "AgcRms"; }
  Dt in_type() const override { return iq_ ? Dt::C32 : Dt::F32; }
  Dt out_type() const override { return iq_ ? Dt::C32 : Dt::F32; }
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const long long n = static_cast<long long>(std::min(n_in, out_cap));  // agc.rs:49
    if (n == 0) return {0, 0};
    // Chunk length 256: >> 1024 waves share the serial W-sample warm-up (envelope only).
    const long long L = warm_ < 0 ? n : 256;
    const long long chunks = (n + L - 1) / L;
    float* e = env_.as<float>();
    float* ein = e + cur_;
    float* eout = e + (cur_ ^ 1);
    const unsigned grid = static_cast<unsigned>((chunks + 255) / 256);
    const float* x = static_cast<const float*>(in);
    float* y = static_cast<float*>(out);
    if (iq_) {
      hipLaunchKernelGGL(k_agc<true>, dim3(grid), dim3(256), 0, s, x, y, n, L, warm_ < 0 ? 0 : warm_, k_, ein, eout);
    } else {
      hipLaunchKernelGGL(k_agc<false>, dim3(grid), dim3(256), 0, s, x, y, n, L, warm_ < 0 ? 0 : warm_, k_, ein, eout);
    }
    ORION_HIP(hipGetLastError());
    cur_ ^= 1;
    return {static_cast<size_t>(n), static_cast<size_t>(n)};
  }
  void reset() override {
    env_.zero();
    cur_ = 0;
  }
  std::vector<float> taps(int) const override {
    return {k_.att, k_.rel, k_.tgt, static_cast<float>(warm_)};
  }

 private:
  bool iq_;
  AgcK k_{};
  long long warm_ = 0;
  DevBuf env_;  // two floats: the carried envelope, ping-ponged per call
  int cur_ = 0;
};

}  // namespace

std::unique_ptr<Block> make_agc(bool iq, float fs, float attack_ms, float release_ms, float target_rms) {
  return std::make_unique<AgcBlock>(iq, fs, attack_ms, release_ms, target_rms);
}

}  // namespace orion
