// scan_blocks.cpp — stateful IIR / demodulator Blocks over the scan kernels.
#include "scan_blocks.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "osc.hpp"
#include "scan.hpp"

namespace orion {
namespace {

// One recurrence stage: rec/pre/post choice, transition matrices, carried state.
class ScanStage {
 public:
  ScanStage(RecK rec, Pre pre, Post post, const StateSpace& ss, const ScanCoef& c, int nch)
      : rec_(rec), pre_(pre), post_(post), c_(c), nch_(nch), S_(ss.S) {
    const auto mats = build_mats(ss);
    mats_.upload(mats.data(), mats.size() * sizeof(double));
    {  // the zero-state end state of a kSpC-sample lane run (k_scan_sp)
      const auto z = build_zmap(ss, kSpC);
      zmap_.upload(z.data(), z.size() * sizeof(float));
    }
    for (auto& c0 : carry_) c0.resize(static_cast<size_t>(nch_) * kScanCarry * sizeof(float));
    // LpDcCascade after an SSB / AM-abs front end: single pass when the LP4
    // forgets its state within the kSpWarm-sample warm-up (SsbProductDemod at
    // 48 kHz: ||A^256|| ~ 1e-20)
    // LpCascade-type stages that forget within one kSpCH chunk: single pass
    if (scan_sp_supported(rec, pre, post)) {
      const auto m = mat_pow(ss.A, ss.S, kSpCH);
      double fro = 0.0;
      for (double v : m) fro += v * v;
      sp1_ok_ = std::sqrt(fro) < 1e-10;
      // the shortest horizon of 2^trs lane runs (kSpC samples each) the stage forgets within
      for (int trs = 3; trs <= 5; ++trs) {
        const auto mw = mat_pow(ss.A, ss.S, static_cast<uint64_t>(kSpC) << trs);
        double fw = 0.0;
        for (double v : mw) fw += v * v;
        if (std::sqrt(fw) < 1e-10) {
          sp1_trs_ = trs;
          break;
        }
      }
    }
    // DcBlocker alone: k_lpdc_sp's DC look-back without the LP4 (pole ~1: no chunk forgets)
    if (rec == RecK::DC && pre == Pre::Real && post == Post::Id) {
      sp_ok_ = true;
      dc_only_ = true;
    }
    if (rec == RecK::LPDC && (pre == Pre::Ssb || pre == Pre::AmAbs || pre == Pre::AmSqrt || pre == Pre::RealLp ||
                              pre == Pre::RealLpSqrt || pre == Pre::RealLpAbs)) {
      const StateSpace lp = lp_cascade_ss(BiquadCoeffs{c.b0, c.b1, c.b2, c.a1, c.a2});
      const auto m = mat_pow(lp.A, 4, kSpWarm);
      double fro = 0.0;
      for (double v : m) fro += v * v;
      sp_ok_ = std::sqrt(fro) < 1e-10;
      if (sp_ok_) {
        const auto ml = build_mats(lp);
        mats_lp_.upload(ml.data(), ml.size() * sizeof(double));
        const auto zl = build_zmap(lp, kLpdcSC);  // k_lpdc_sp's LP4 lane runs
        zmap_lp_.upload(zl.data(), zl.size() * sizeof(float));
      }
    }
  }
  // sum_i A^(C-1-i) B x_i, the zero-state end state of a C-sample lane run: [C][S] floats
  static std::vector<float> build_zmap(const StateSpace& ss, int C) {
    const int S = ss.S;
    std::vector<float> z(static_cast<size_t>(C) * S, 0.0f);
    std::vector<double> col = ss.B;  // A^j B, j = 0, 1, ...
    if (col.size() != static_cast<size_t>(S)) col.assign(S, 0.0);
    for (int i = C - 1; i >= 0; --i) {
      for (int k = 0; k < S; ++k) z[static_cast<size_t>(i) * S + k] = static_cast<float>(col[k]);
      std::vector<double> nx(S, 0.0);
      for (int r = 0; r < S; ++r)
        for (int k = 0; k < S; ++k) nx[r] += ss.A[r * S + k] * col[k];
      col = nx;
    }
    return z;
  }
  static std::vector<double> build_mats(const StateSpace& ss) {
    const int S = ss.S;
    std::vector<double> mats(static_cast<size_t>(ScanMatsLayout::kCount) * S * S, 0.0);
    auto put = [&](int idx, const std::vector<double>& m) {
      std::copy(m.begin(), m.end(), mats.begin() + static_cast<size_t>(idx) * S * S);
    };
    const auto Mc = mat_pow(ss.A, S, kScanC);
    auto p = Mc;
    for (int s = 0; s < 6; ++s) {
      put(ScanMatsLayout::kPwc + s, p);
      p = mat_mul(p, p, S);
    }
    put(ScanMatsLayout::kM64, mat_pow(ss.A, S, 64ull * kScanC));
    put(ScanMatsLayout::kM128, mat_pow(ss.A, S, 128ull * kScanC));
    p = mat_pow(ss.A, S, kScanCH);
    for (int s = 0; s < 8; ++s) {
      put(ScanMatsLayout::kPch + s, p);
      p = mat_mul(p, p, S);
    }
    for (int L = 0; L < 64; ++L) put(ScanMatsLayout::kLane + L, mat_pow(ss.A, S, static_cast<uint64_t>(kScanC) * L));
    return mats;
  }
  // 0 auto (single pass where valid), 1 force the three-kernel scan (tests)
  void set_mode(int m) { mode_ = m; }
  bool lpdc_single_pass() const { return sp_ok_; }
  // The stage's Rotator (the SSB BFO, ssb.rs:18; the FM translator, fm.rs:35): the
  // reference recurrence, tabulated (osc.hpp RefOsc); its outputs advance with the samples.
  void set_osc(float freq_hz, float fs) { osc_ = std::make_unique<RefOsc>(freq_hz, fs); }
  RefOsc* osc() { return osc_.get(); }
  void reset_osc() {
    if (osc_) osc_->reset();
  }
  void set_carry(const std::vector<float>& per_ch) {  // kScanCarry floats, same for every channel
    std::vector<float> c(static_cast<size_t>(nch_) * kScanCarry);
    for (int ch = 0; ch < nch_; ++ch) std::copy(per_ch.begin(), per_ch.end(), c.begin() + ch * kScanCarry);
    for (auto& c0 : carry_) c0.upload(c.data(), c.size() * sizeof(float));
    cur_ = 0;
  }
  ScanCoef& coef() { return c_; }
  void set_translate(bool on) { translate_ = on; }
  void run(const void* x, long long x_stride, long long n, void* y, long long y_stride, long long k0,
           int* err, hipStream_t s) {
    const long long nblk = (n + kScanCH - 1) / kScanCH;
    ws_.resize(static_cast<size_t>(2 * nblk * nch_ * S_ + 16) * sizeof(double));
    ScanArgs a{};
    a.x = x;
    a.x_stride = x_stride;
    a.y = y;
    a.y_stride = y_stride;
    a.n = n;
    a.k0 = osc_ ? static_cast<long long>(osc_->count()) : k0;
    a.translate = translate_ ? 1 : 0;
    if (osc_) a.osc = osc_->dev(static_cast<uint64_t>(n), s);
    a.mats = mats_.as<double>();
    a.zmap = sp1_ok_ || !sp_ok_ ? zmap_.as<float>() : zmap_lp_.as<float>();  // k_lpdc_sp: its LP4's map
    a.aggs = ws_.as<double>();
    a.sin = ws_.as<double>() + nblk * nch_ * S_;
    a.carry_in = carry_[cur_].as<float>();
    a.carry_out = carry_[cur_ ^ 1].as<float>();
    a.c = c_;
    a.err = err;
    a.spin = spin_limit();
    if ((sp_ok_ || sp1_ok_) && mode_ == 0) {
      const size_t words = sp1_ok_ ? static_cast<size_t>(scan_sp_chunks(n)) * nch_ * 16
                                   : static_cast<size_t>(lpdc_sp_demod_chunks(n, kLpdcSC, dc_only_ ? 0 : kSpWarm)) * nch_ * 8;
      if (words * 4 > rec_buf_.size()) {
        rec_buf_.resize(words * 4);
        rec_buf_.zero(s);
        epoch_ = 0;
      }
      if (++epoch_ == 0xFFFFFFFFu) {  // never reuse a tag that may sit in a record
        rec_buf_.zero(s);
        epoch_ = 1;
      }
      if (sp1_ok_) launch_scan_sp(rec_, pre_, post_, a, nch_, rec_buf_.as<uint32_t>(), epoch_, sp1_trs_, s);
      else launch_lpdc_sp(pre_, a, mats_lp_.as<double>(), nch_, rec_buf_.as<uint32_t>(), epoch_, s);
    } else {
      launch_scan(rec_, pre_, post_, a, nch_, s);
    }
    if (osc_) osc_->advance(static_cast<uint64_t>(n));
    cur_ ^= 1;
  }

 private:
  RecK rec_;
  Pre pre_;
  Post post_;
  ScanCoef c_;
  int nch_, S_;
  bool translate_ = false;
  std::unique_ptr<RefOsc> osc_;
  DevBuf mats_, carry_[2], ws_, mats_lp_, rec_buf_, zmap_, zmap_lp_;
  int cur_ = 0;
  bool sp_ok_ = false;   // k_lpdc_sp (LpDcCascade after SSB / AM-abs)
  bool sp1_ok_ = false;  // k_scan_sp (stages that forget within one chunk)
  bool dc_only_ = false;  // k_lpdc_sp<Real>: the DcBlocker alone
  int sp1_trs_ = 0;  // k_scan_sp lane scan truncated to 2^sp1_trs_ lane runs (0: full)
  int mode_ = 0;
  uint32_t epoch_ = 0;
};

ScanCoef coef_lp(const BiquadCoeffs& b) {
  ScanCoef c{};
  c.b0 = b.b0; c.b1 = b.b1; c.b2 = b.b2; c.a1 = b.a1; c.a2 = b.a2;
  return c;
}

// Generic single-stage f32/cf32 -> f32 block.
class ScanBlock : public Block {
 public:
  ScanBlock(const char* nm, Dt in, int nch) : nm_(nm), in_(in), nch_(nch) {}
  const char* name() const override { return nm_; }
  Dt in_type() const override { return in_; }
  Dt out_type() const override { return Dt::F32; }
  int channels() const override { return nch_; }
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const size_t n = std::min(n_in, out_cap);  // 1:1 blocks: min(in, out)
    if (n == 0) return {0, 0};
    run(in, n_in, n, out, out_cap, s);
    k0_ += n;
    return {n, n};
  }
  void reset() override {
    k0_ = 0;
    reset_state();
    ORION_HIP(hipDeviceSynchronize());
  }

 protected:
  virtual void run(const void* in, size_t stride, size_t n, void* out, size_t out_stride, hipStream_t s) = 0;
  virtual void reset_state() = 0;
  const char* nm_;
  Dt in_;
  int nch_;
  uint64_t k0_ = 0;
};

class OneStageBlock : public ScanBlock {
 public:
  OneStageBlock(const char* nm, Dt in, int nch, std::unique_ptr<ScanStage> st, std::vector<float> carry0)
      : ScanBlock(nm, in, nch), st_(std::move(st)), carry0_(std::move(carry0)) {
    reset_state();
  }
  ScanStage& stage() { return *st_; }
  std::vector<float> taps(int) const override { return coef_; }
  int configure(int option, long long value) override {
    if (option == kOptNcoTable && st_->osc()) {  // the BFO / translator Rotator's table budget
      if (value < 0 || static_cast<unsigned long long>(value) > kNcoTableMax) return -3;
      st_->osc()->set_budget(static_cast<uint64_t>(value));
      return 0;
    }
    if (option != kOptScanPath) return -4;
    if (value != 0 && value != 1) return -3;
    st_->set_mode(static_cast<int>(value));
    return 0;
  }
  std::vector<float> coef_;

 protected:
  void run(const void* in, size_t stride, size_t n, void* out, size_t out_stride, hipStream_t s) override {
    st_->run(in, static_cast<long long>(stride), static_cast<long long>(n), out, static_cast<long long>(out_stride),
             static_cast<long long>(k0_), dev_err(), s);
  }
  void reset_state() override {
    st_->set_carry(carry0_);
    st_->reset_osc();
  }
  std::unique_ptr<ScanStage> st_;
  std::vector<float> carry0_;
};

std::vector<float> carry_zero() { return std::vector<float>(kScanCarry, 0.0f); }
std::vector<float> carry_prev_one() {  // FM/PM: prev = 1 + 0j (fm.rs:29, pm.rs:31)
  auto c = carry_zero();
  c[6] = 1.0f;
  return c;
}

// AM envelope: PowerSqrt = LP4 -> sqrt -> DC (two scans through a temp buffer);
// AbsApprox = one LpDc scan.
class AmBlock final : public ScanBlock {
 public:
  AmBlock(float fs, float bw) : ScanBlock("AmEnvelopeDemod", Dt::C32, 1) {
    d_ = lpdc_design(fs, bw * 0.9f, 2.0f);  // am.rs:27
    ScanCoef c = coef_lp(d_.bq);
    c.r = d_.r;
    lp_ = std::make_unique<ScanStage>(RecK::LP4, Pre::AmSqrt, Post::Sqrt, lp_cascade_ss(d_.bq), c, 1);
    dc_ = std::make_unique<ScanStage>(RecK::DC, Pre::Real, Post::Id, dc_ss(d_.r), c, 1);
    lpdc_ = std::make_unique<ScanStage>(RecK::LPDC, Pre::AmAbs, Post::Id, lpdc_ss(d_), c, 1);
    // PowerSqrt in one pass (k_lpdc_sp with the sqrt between the LP4 and the DC
    // blocker) when the LP4 forgets within the warm-up; otherwise the two scans
    sq_ = std::make_unique<ScanStage>(RecK::LPDC, Pre::AmSqrt, Post::Id, lpdc_ss(d_), c, 1);
    if (!sq_->lpdc_single_pass()) sq_.reset();
    reset_state();
  }
  int configure(int option, long long value) override {
    if (option != kOptScanPath) return -4;
    if (value != 0 && value != 1) return -3;
    for (auto* st : {lp_.get(), dc_.get(), lpdc_.get()}) st->set_mode(static_cast<int>(value));
    three_ = value == 1;
    return 0;
  }
  void set_abs(float k1, float k2) {
    abs_ = true;
    lpdc_->coef().k1 = k1;
    lpdc_->coef().k2 = k2;
  }
  std::vector<float> taps(int) const override {
    return {d_.bq.b0, d_.bq.b1, d_.bq.b2, d_.bq.a1, d_.bq.a2, d_.r};
  }

 protected:
  void run(const void* in, size_t stride, size_t n, void* out, size_t out_stride, hipStream_t s) override {
    if (abs_) {
      lpdc_->run(in, static_cast<long long>(stride), static_cast<long long>(n), out, static_cast<long long>(out_stride),
                 static_cast<long long>(k0_), dev_err(), s);
      return;
    }
    if (sq_ && !three_) {
      sq_->run(in, static_cast<long long>(stride), static_cast<long long>(n), out, static_cast<long long>(out_stride),
               static_cast<long long>(k0_), dev_err(), s);
      return;
    }
    tmp_.resize(n * sizeof(float) + 16);
    lp_->run(in, static_cast<long long>(stride), static_cast<long long>(n), tmp_.as<void>(), static_cast<long long>(n),
             static_cast<long long>(k0_), dev_err(), s);
    dc_->run(tmp_.as<void>(), static_cast<long long>(n), static_cast<long long>(n), out,
             static_cast<long long>(out_stride), static_cast<long long>(k0_), dev_err(), s);
  }
  void reset_state() override {
    lp_->set_carry(carry_zero());
    dc_->set_carry(carry_zero());
    lpdc_->set_carry(carry_zero());
    if (sq_) sq_->set_carry(carry_zero());
  }

 private:
  LpDcCoeffs d_;
  bool abs_ = false, three_ = false;
  std::unique_ptr<ScanStage> lp_, dc_, lpdc_, sq_;
  DevBuf tmp_;
};

// dsp/iir.rs:86-187 LpDcCascade as an f32 block: process (LP4 -> DC blocker) or
// process_mapped(x, f) (LP4 -> f -> DC) with f one of the maps the ABI names: identity
// (== process), f32::sqrt (the AM-PowerSqrt use, am.rs:55) or f32::abs.
// One pass (k_lpdc_sp<RealLp / RealLpSqrt / RealLpAbs>) when the LP4 forgets within the
// warm-up; otherwise the three-kernel LpDc scan, or (sqrt / abs) an LP4 scan with the map
// as its post-stage and a DC scan.
class LpDcBlock final : public ScanBlock {
 public:
  LpDcBlock(float fs, float lp_fc, float dc_cut) : ScanBlock("LpDcCascade", Dt::F32, 1) {
    d_ = lpdc_design(fs, lp_fc, dc_cut);  // iir.rs:111-137
    ScanCoef c = coef_lp(d_.bq);
    c.r = d_.r;
    sp_ = std::make_unique<ScanStage>(RecK::LPDC, Pre::RealLp, Post::Id, lpdc_ss(d_), c, 1);
    sq_ = std::make_unique<ScanStage>(RecK::LPDC, Pre::RealLpSqrt, Post::Id, lpdc_ss(d_), c, 1);
    ab_ = std::make_unique<ScanStage>(RecK::LPDC, Pre::RealLpAbs, Post::Id, lpdc_ss(d_), c, 1);
    full_ = std::make_unique<ScanStage>(RecK::LPDC, Pre::Real, Post::Id, lpdc_ss(d_), c, 1);
    lp_ = std::make_unique<ScanStage>(RecK::LP4, Pre::Real, Post::Sqrt, lp_cascade_ss(d_.bq), c, 1);
    lpa_ = std::make_unique<ScanStage>(RecK::LP4, Pre::Real, Post::Abs, lp_cascade_ss(d_.bq), c, 1);
    dc_ = std::make_unique<ScanStage>(RecK::DC, Pre::Real, Post::Id, dc_ss(d_.r), c, 1);
    reset_state();
  }
  // process_mapped with map (kMapIdentity / kMapSqrt / kMapAbs, iir.rs:170-186) from now
  // on: before the first call. Identity is process itself (:151-165 == :170-186 with |v| v).
  void set_map(int map) { map_ = map; }
  int configure(int option, long long value) override {
    if (option != kOptScanPath) return -4;
    if (value != 0 && value != 1) return -3;
    three_ = value == 1;
    for (auto* st : {lp_.get(), lpa_.get(), dc_.get(), full_.get()}) st->set_mode(static_cast<int>(value));
    return 0;
  }
  std::vector<float> taps(int) const override { return {d_.bq.b0, d_.bq.b1, d_.bq.b2, d_.bq.a1, d_.bq.a2, d_.r}; }

 protected:
  void run(const void* in, size_t stride, size_t n, void* out, size_t out_stride, hipStream_t s) override {
    const long long st = static_cast<long long>(stride), nn = static_cast<long long>(n),
                    os = static_cast<long long>(out_stride), k0 = static_cast<long long>(k0_);
    if (map_ == kMapIdentity) {
      if (sp_->lpdc_single_pass() && !three_) sp_->run(in, st, nn, out, os, k0, dev_err(), s);
      else full_->run(in, st, nn, out, os, k0, dev_err(), s);
      return;
    }
    ScanStage* one = map_ == kMapSqrt ? sq_.get() : ab_.get();
    if (one->lpdc_single_pass() && !three_) {
      one->run(in, st, nn, out, os, k0, dev_err(), s);
      return;
    }
    tmp_.resize(n * sizeof(float) + 16);
    (map_ == kMapSqrt ? lp_ : lpa_)->run(in, st, nn, tmp_.as<void>(), nn, k0, dev_err(), s);
    dc_->run(tmp_.as<void>(), nn, nn, out, os, k0, dev_err(), s);
  }
  void reset_state() override {
    for (auto* st : {sp_.get(), sq_.get(), ab_.get(), full_.get(), lp_.get(), lpa_.get(), dc_.get()})
      st->set_carry(carry_zero());
  }

 private:
  LpDcCoeffs d_;
  int map_ = kMapIdentity;
  bool three_ = false;
  std::unique_ptr<ScanStage> sp_, sq_, ab_, full_, lp_, lpa_, dc_;
  DevBuf tmp_;
};

// modulate/ssb.rs:9-114. F32 audio -> C32 IQ: the audio-NCO products (k_mod), both
// LpCascades as one 2-channel LP4 scan (I, Q planar), then (I, side Q) x RF NCO.
class SsbModBlock final : public Block {
 public:
  SsbModBlock(float fs, float bw, float if_hz, float rf_hz, bool usb)
      : aud_(if_hz, fs), rf_(rf_hz, fs), side_(usb ? 1.0f : -1.0f) {  // ssb.rs:32-33: two Rotators
    b_ = lp_cascade_design(fs, bw * 0.9f);  // ssb.rs:25
    const StateSpace ss = lp_cascade_ss(b_);
    st_ = std::make_unique<ScanStage>(RecK::LP4, Pre::Real, Post::Id, ss, coef_lp(b_), 2);
    st_->set_carry(carry_zero());
    // one pass when the LP4 forgets its state within the kSpWarm-sample warm-up
    const auto m = mat_pow(ss.A, 4, kSpWarm);
    double fro = 0.0;
    for (double v : m) fro += v * v;
    sp_ok_ = std::sqrt(fro) < 1e-10;
    if (sp_ok_) {
      const auto ml = ScanStage::build_mats(ss);
      mats_.upload(ml.data(), ml.size() * sizeof(double));
      const auto zl = ScanStage::build_zmap(ss, kScanC);  // k_ssb_mod_sp's lane runs
      zmap_.upload(zl.data(), zl.size() * sizeof(float));
      for (auto& c : carry_) c.resize(8 * sizeof(float));
    }
    reset_sp();
  }
  const char* name() const override { return "SsbPhasingMod"; }
  Dt in_type() const override { return Dt::F32; }
  Dt out_type() const override { return Dt::C32; }
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const size_t n = std::min(n_in, out_cap);  // ssb.rs:44
    if (n == 0) return {0, 0};
    const long long nn = static_cast<long long>(n);
    if (sp_ok_ && mode_ == 0) {
      launch_ssb_mod_sp(static_cast<const float*>(in), static_cast<f2*>(out), nn, aud_.count(), aud_.dev(n, s), rf_.dev(n, s),
                        side_, coef_lp(b_), mats_.as<double>(), zmap_.as<float>(), carry_[cur_].as<float>(),
                        carry_[cur_ ^ 1].as<float>(), s);
      cur_ ^= 1;
    } else {
      u_.resize(2 * n * sizeof(float));
      v_.resize(2 * n * sizeof(float));
      launch_ssb_mod_front(static_cast<const float*>(in), u_.as<float>(), nn, aud_.count(), aud_.dev(n, s), s);
      st_->run(u_.as<void>(), nn, nn, v_.as<void>(), nn, 0, dev_err(), s);
      launch_ssb_mod_back(v_.as<float>(), static_cast<f2*>(out), nn, rf_.count(), rf_.dev(n, s), side_, s);
    }
    aud_.advance(n);
    rf_.advance(n);
    return {n, n};
  }
  void reset() override {
    aud_.reset();
    rf_.reset();
    st_->set_carry(carry_zero());
    reset_sp();
    ORION_HIP(hipDeviceSynchronize());
  }
  int configure(int option, long long value) override {  // single pass where valid, or the three passes
    if (option == kOptNcoTable) {  // both Rotators' table budgets
      if (value < 0 || static_cast<unsigned long long>(value) > kNcoTableMax) return -3;
      aud_.set_budget(static_cast<uint64_t>(value));
      rf_.set_budget(static_cast<uint64_t>(value));
      return 0;
    }
    if (option != kOptModPasses) return -4;
    if (value != 0 && value != 1 && value != 3) return -3;
    mode_ = value == 3 ? 1 : 0;
    return 0;
  }
  std::vector<float> taps(int) const override { return {b_.b0, b_.b1, b_.b2, b_.a1, b_.a2}; }

 private:
  void reset_sp() {
    if (!sp_ok_) return;
    const std::vector<float> z(8, 0.0f);
    for (auto& c : carry_) c.upload(z.data(), z.size() * sizeof(float));
    cur_ = 0;
  }
  RefOsc aud_, rf_;
  float side_;
  BiquadCoeffs b_;
  std::unique_ptr<ScanStage> st_;
  DevBuf u_, v_, mats_, carry_[2], zmap_;
  bool sp_ok_ = false;
  int mode_ = 0, cur_ = 0;
};

}  // namespace

std::unique_ptr<Block> make_ssb_mod(float fs, float audio_bw, float audio_if_hz, float rf_hz, bool usb) {
  return std::make_unique<SsbModBlock>(fs, audio_bw, audio_if_hz, rf_hz, usb);
}

std::unique_ptr<Block> make_lp_cascade(float fs, float fc) {
  const BiquadCoeffs b = lp_cascade_design(fs, fc);
  auto st = std::make_unique<ScanStage>(RecK::LP4, Pre::Real, Post::Id, lp_cascade_ss(b), coef_lp(b), 1);
  auto blk = std::make_unique<OneStageBlock>("LpCascade", Dt::F32, 1, std::move(st), carry_zero());
  blk->coef_ = {b.b0, b.b1, b.b2, b.a1, b.a2};
  return blk;
}

std::unique_ptr<Block> make_biquad(float b0, float b1, float b2, float a1, float a2) {
  const BiquadCoeffs b{b0, b1, b2, a1, a2};  // iir.rs:17-27
  auto st = std::make_unique<ScanStage>(RecK::BQ, Pre::Real, Post::Id, biquad_ss(b), coef_lp(b), 1);
  auto blk = std::make_unique<OneStageBlock>("Biquad", Dt::F32, 1, std::move(st), carry_zero());
  blk->coef_ = {b0, b1, b2, a1, a2};
  return blk;
}

std::unique_ptr<Block> make_lp_dc_cascade(float fs, float lp_fc, float dc_cut_hz) {
  return std::make_unique<LpDcBlock>(fs, lp_fc, dc_cut_hz);
}

int lp_dc_cascade_set_map(Block* b, int map) {
  auto* l = dynamic_cast<LpDcBlock*>(b);
  if (!l) return -4;
  if (map != kMapIdentity && map != kMapSqrt && map != kMapAbs) return -3;
  l->set_map(map);
  return 0;
}

std::unique_ptr<Block> make_dc_blocker(float fs, float cut_hz) {
  const float r = dc_blocker_pole(fs, cut_hz);
  ScanCoef c{};
  c.r = r;
  auto st = std::make_unique<ScanStage>(RecK::DC, Pre::Real, Post::Id, dc_ss(r), c, 1);
  auto blk = std::make_unique<OneStageBlock>("DcBlocker", Dt::F32, 1, std::move(st), carry_zero());
  blk->coef_ = {r};
  return blk;
}

std::unique_ptr<Block> make_fm_demod(float fs, float dev_hz, float audio_bw) {
  const BiquadCoeffs b = lp_cascade_design(fs, audio_bw * 0.9f);  // fm.rs:24
  ScanCoef c = coef_lp(b);
  c.k = 1.0f / std::max(dev_hz, 1.0f);  // fm.rs:23
  auto st = std::make_unique<ScanStage>(RecK::LP4, Pre::Fm, Post::Id, lp_cascade_ss(b), c, 1);
  auto blk = std::make_unique<OneStageBlock>("FmQuadratureDemod", Dt::C32, 1, std::move(st), carry_prev_one());
  blk->coef_ = {b.b0, b.b1, b.b2, b.a1, b.a2, c.k, fs};
  return blk;
}

int fm_demod_with_translate(Block* b, float freq_hz) {
  auto* o = dynamic_cast<OneStageBlock*>(b);
  if (!o || std::strcmp(b->name(), "FmQuadratureDemod") != 0) return -4;
  o->stage().set_osc(freq_hz, o->coef_[6]);  // Rotator::new(freq_hz, fs), fm.rs:35
  o->stage().set_translate(true);
  return 0;
}

std::unique_ptr<Block> make_pm_demod(float fs, float k, float audio_bw) {
  const BiquadCoeffs b = lp_cascade_design(fs, audio_bw * 0.9f);  // pm.rs:27
  ScanCoef c = coef_lp(b);
  c.k = k;
  auto st = std::make_unique<ScanStage>(RecK::LP4, Pre::Pm, Post::Id, lp_cascade_ss(b), c, 1);
  auto blk = std::make_unique<OneStageBlock>("PmQuadratureDemod", Dt::C32, 1, std::move(st), carry_prev_one());
  blk->coef_ = {b.b0, b.b1, b.b2, b.a1, b.a2, k};
  return blk;
}

std::unique_ptr<Block> make_ssb_demod(float fs, float bfo_hz, float audio_bw, int nch) {
  const LpDcCoeffs d = lpdc_design(fs, audio_bw * 0.9f, 2.0f);  // ssb.rs:17
  ScanCoef c = coef_lp(d.bq);
  c.r = d.r;
  auto st = std::make_unique<ScanStage>(RecK::LPDC, Pre::Ssb, Post::Id, lpdc_ss(d), c, nch);
  st->set_osc(bfo_hz, fs);  // ssb.rs:18 Rotator::new(bfo_hz, fs)
  auto blk = std::make_unique<OneStageBlock>("SsbProductDemod", Dt::C32, nch, std::move(st), carry_zero());
  blk->coef_ = {d.bq.b0, d.bq.b1, d.bq.b2, d.bq.a1, d.bq.a2, d.r};
  return blk;
}

std::unique_ptr<Block> make_am_demod(float fs, float audio_bw) { return std::make_unique<AmBlock>(fs, audio_bw); }

int am_demod_with_abs_approx(Block* b, float k1, float k2) {
  auto* a = dynamic_cast<AmBlock*>(b);
  if (!a) return -4;
  a->set_abs(k1, k2);
  return 0;
}

std::unique_ptr<Block> make_cw_demod(float fs, float tone_hz, float env_bw) {
  (void)tone_hz;  // cw.rs:15: accepted for API symmetry, unused
  const float a = cw_alpha(fs, env_bw);
  ScanCoef c{};
  c.a = a;
  c.gain = 1.0f;
  auto st = std::make_unique<ScanStage>(RecK::ONEPOLE, Pre::Cw, Post::Gain, onepole_ss(a), c, 1);
  auto blk = std::make_unique<OneStageBlock>("CwEnvelopeDemod", Dt::C32, 1, std::move(st), carry_zero());
  blk->coef_ = {a};
  return blk;
}

int cw_demod_set_gain(Block* b, float g) {
  auto* o = dynamic_cast<OneStageBlock*>(b);
  if (!o || std::strcmp(b->name(), "CwEnvelopeDemod") != 0) return -4;
  o->stage().coef().gain = g;
  return 0;
}

}  // namespace orion
