// scan_blocks.hpp — Blocks built on the state-carry scan (scan.hpp).
#pragma once
#include <memory>

#include "blocks.hpp"

namespace orion {

std::unique_ptr<Block> make_lp_cascade(float fs, float fc);                  // dsp/iir.rs:49-83
std::unique_ptr<Block> make_biquad(float b0, float b1, float b2, float a1, float a2);  // dsp/iir.rs:15-41
std::unique_ptr<Block> make_lp_dc_cascade(float fs, float lp_fc, float dc_cut_hz);     // dsp/iir.rs:86-187
// process_mapped(x, f) (iir.rs:170-186) with f = identity / f32::sqrt / f32::abs
// (include/orion_sdr_amd.h ORION_MAP_*); -4 other blocks, -3 an unknown map.
enum : int { kMapIdentity = 0, kMapSqrt = 1, kMapAbs = 2 };
int lp_dc_cascade_set_map(Block* b, int map);
// modulate/ssb.rs:9-114 (SsbPhasingMod::new(fs, audio_bw, audio_if, rf, usb)). F32 -> C32.
std::unique_ptr<Block> make_ssb_mod(float fs, float audio_bw, float audio_if_hz, float rf_hz, bool usb);
std::unique_ptr<Block> make_dc_blocker(float fs, float cut_hz);              // dsp/dc.rs:8-59
std::unique_ptr<Block> make_fm_demod(float fs, float dev_hz, float audio_bw);  // demodulate/fm.rs
int fm_demod_with_translate(Block* b, float freq_hz);                        // fm.rs:34-37
std::unique_ptr<Block> make_pm_demod(float fs, float k, float audio_bw);     // demodulate/pm.rs
std::unique_ptr<Block> make_ssb_demod(float fs, float bfo_hz, float audio_bw, int nch);  // ssb.rs
std::unique_ptr<Block> make_am_demod(float fs, float audio_bw);              // demodulate/am.rs
int am_demod_with_abs_approx(Block* b, float k1, float k2);                  // am.rs:33-36
std::unique_ptr<Block> make_cw_demod(float fs, float tone_hz, float env_bw);  // demodulate/cw.rs
int cw_demod_set_gain(Block* b, float g);                                    // cw.rs:26-28

}  // namespace orion
