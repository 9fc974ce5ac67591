// Internal interface (not exported) between fvc_conv_x3.hip's host dispatcher and the
// all-classes transposed-conv kernel of fvc_deconv_x3.hip.
#pragma once
#include "fvc_common.h"

namespace fvc_dx {

constexpr int kMaxTaps = 9;  // taps per parity class (5x5 stride 2: 9, 6, 6, 4)
constexpr int kWaves = 8;
constexpr int kMaxWT = 4;    // wave-tiles per wave per work item

struct DxArgs {
  const float* x;     // [B][H][W][cinp] fp32
  const uint4* w;     // x3 pack with one channel chunk: [class][k-step][N-tile][hi|lo][lane]
  const float* bias;
  const float* res;   // residual [B][2H][2W][coutp] or null (plain epilogue only)
  float* y;           // [B][2H][2W][coutp], or tap partials [B][2H][2W][pcp]
  int post_exp;       // exp after the residual (pad channels 0)
  int B, H, W, cout, coutp, ntp;
  int R;              // input rows per work item
  int sw;             // input columns per work item = pixels per strip row (32: 1 x 32 strips, 16: 2 x 16)
  int ir, ic, ps;     // staged tile rows / columns, LDS plane stride (16-B entries, odd)
  int dymin, dxmin;
  float inv_ic;
  int tiles_x, tiles_y, nitems;
  float osc, osc_c, act_slope;
  int nks[4];                    // k-steps per class (taps x cinp / 16)
  int oy0[4], ox0[4];            // output parity of each class
  long long wcls[4];             // uint4 offset of each class in the pack
  int toff[4][kMaxTaps + 1];     // LDS pixel offset of each tap's window, per class
  int wt[kWaves][kMaxWT];        // wave-tiles per wave: class | first strip << 4 | first N-tile << 8; -1 ends
  unsigned y_bytes, x_bytes;     // descriptor ranges (< 4 GB, checked by the caller)
  int* sched;                    // [0] blocks done, [1] next item: zero on entry, reset by the last block
  int* ovf;
  const uint4* tw;               // tap epilogue: packed partial weights (fvc_x3_tap_pack_weight)
  float tosc, tosc_c;
  int pcp;
};

// LDS bytes of one launch (header + two full-channel tile buffers)
__attribute__((visibility("hidden"))) size_t lds_bytes(int cinp, int ps);
// odd plane stride >= ir * ic (conflict-free staging writes of consecutive octets)
__attribute__((visibility("hidden"))) int plane_pix(int ir, int ic);
// strip width of a geometry: 16 (2 x 16-pixel strips, 8-row items) for 128 input channels, else 32
inline int strip_width(int cinp) { return cinp == 128 ? 16 : 32; }
// cinp in {64, 96, 128}; (wm, wn) = (2, 2) plain epilogue or (1, ntp) with the tap epilogue;
// iop in {FVC_IN_NONE, FVC_IN_ROUND}
__attribute__((visibility("hidden"))) int launch(const DxArgs& a, int cinp, int wm, int wn, int iop, bool tap,
                                                 int grid, size_t lds, hipStream_t s);

}  // namespace fvc_dx
