// Named kernel-configuration slots: the A/B switches and the autotuner's overrides that select
// kernel variants at launch time (g_tune[slot], 0 = the shipped heuristic).  The names are the
// interface: Python addresses slots only through ddp_classification_pytorch_amd/tuning.py, which
// mirrors this table (tests/test_tuning_cpu.py checks the two agree; _ext checks the loaded
// library's table at load time), and DCP_TUNE="name=value,..." sets them from the environment.
#pragma once

namespace dcp {

enum TuneSlot : int {
  kTgTileN = 0,        // tap GEMM output-channel tile: 64 / 128 / 256
  kTgStages = 1,       // tap GEMM LDS stages (2..4)
  kAblate = 2,         // timing ablations (tap GEMM, direct 3x3): 1 no staging / stores, 2 no MFMA / window loads
  kTgPingPong = 3,     // ping-pong 256-row tap GEMM: 1 on where it applies, 2 off (0 = heuristic)
  kTgBigCvar = 4,      // big-tile tap GEMM compute variant: 2 = fragments read after the barrier
  kWgSplitsPerCu = 5,  // weight gradient: split-K workgroups per CU
  kWgFlushAblate = 6,  // weight gradient: 1 = time the atomic flush only (dW not zeroed)
  kWgTileMode = 7,     // weight gradient: 2 = no 256-column kernel, 3 = no 64-row kernel
  kTgKDepth = 8,       // tap GEMM k-tile depth: 32 / 64 (64 also disables the 1x1 32-deep rule)
  kEwGridCap = 9,      // BN elementwise kernels: workgroup cap
  kEwRows = 10,        // BN elementwise kernels: rows per thread
  kBnActVariant = 11,  // BN apply (+ReLU) kernel variant
  kWgRows = 12,        // weight gradient: 32 = 32-row k-tiles
  kNarrowKDepth = 13,  // narrow-channel (per-lane tap) tap GEMM k-tile depth: 32 / 64
  kWgCols = 14,        // weight gradient column tile: 4 = 256, 3 = 192
  kWg3x3 = 15,         // direct 3x3 weight gradient: 1 off, 2 forced on every pair count
  kGconvSG = 16,       // grouped conv weight gradient: 32 = 32-channel super-groups, 1 = general tap path
  kStemAblate = 17,    // stem timing ablations: 1 no MFMA phase, 2 no gather phase
  kC3Off = 18,         // direct 64->64 3x3: 1 = the implicit GEMM instead
  kC3Variant = 19,     // direct 64->64 3x3 workgroup variant (0 = 8 waves, 1 / 2 = 4-wave, 3 / 4 = priority / phase)
  kDgradParityStreams = 20,  // stride-2 data gradient: 1 = the four parity classes on concurrent streams
  kTgBigPersist = 22,  // 256-row big tiles: 1 = persistent workgroups (one per CU, looping over tiles)
  kTgBigSK = 23,       // 256-row big tiles, stream-K (k-steps split evenly over one workgroup per CU slot): 1 on, 2 off
  kTgBigStages = 21,   // 256 x 256 big tile: LDS-DMA ring slots (0 = 4; 5 = all 160 KB, three k-tiles in flight)
  kGconvSpw = 26,     // grouped conv fwd / dgrad: super-groups per workgroup (1 = one per workgroup)
  kTgBig = 24,         // big-tile tap GEMM: 1 on (256 x 256 / 256 x 128), 2 off, 3 = 256 x 128 only
  kAutotune = 25,      // per-shape autotuning of the conv configurations (DCP_AUTOTUNE)
  kWgSplitCap = 27,    // weight gradient: at most this many split-K partials
  kBnBwdCap = 28,      // BN-backward reduction workgroup cap
  kRowReduce = 29,     // narrow split reduction in one launch: 2 off, > 2 depth limit
  kC3Epilogue = 30,    // direct 64->64 3x3 epilogue: 2 = LDS-staged (default: from the accumulators)
  kC3WindowKB = 31,    // direct 64->64 3x3 window buffer size (KB)
  kTgWs = 32,          // 1x1 stride-1 short-K forward: 1 = weight-stationary persistent kernel (conv_ws.hip), 2 = off
  kTgPs = 33,          // 1x1 stride-1 short-K forward: store-decoupled loader/consumer kernel (conv1x1_ps.hip), 1 = 4 / 3 = 8 consumer waves, 2 = off
  kBnFinAct = 34,      // the bn_fin_act op (opt-in from Python, DCP_BN_FIN_ACT=1): 2 = run it as its two launches
  kTgSplitK = 35,      // 128-row tap GEMM split-K for short grids with deep k-loops: 2 off, >= 3 slices (A/B), 0 heuristic
  kTuneSlots = 40
};

struct TuneSlotName {
  const char* name;
  int slot;
};

constexpr TuneSlotName kTuneSlotNames[] = {
    {"tg_tile_n", kTgTileN},         {"tg_stages", kTgStages},       {"ablate", kAblate},
    {"tg_pingpong", kTgPingPong},    {"tg_big_cvar", kTgBigCvar},    {"wg_splits_per_cu", kWgSplitsPerCu},
    {"wg_flush_ablate", kWgFlushAblate}, {"wg_tile_mode", kWgTileMode}, {"tg_kdepth", kTgKDepth},
    {"ew_grid_cap", kEwGridCap},     {"ew_rows", kEwRows},           {"bn_act_variant", kBnActVariant},
    {"wg_rows", kWgRows},            {"narrow_kdepth", kNarrowKDepth}, {"wg_cols", kWgCols},
    {"wg3x3", kWg3x3},               {"gconv_sg", kGconvSG},         {"stem_ablate", kStemAblate},
    {"c3_off", kC3Off},              {"c3_variant", kC3Variant},     {"tg_big", kTgBig},
    {"dgrad_parity_streams", kDgradParityStreams}, {"tg_big_stages", kTgBigStages},
    {"tg_big_persist", kTgBigPersist}, {"tg_big_sk", kTgBigSK},
    {"gconv_spw", kGconvSpw},
    {"autotune", kAutotune},         {"wg_split_cap", kWgSplitCap},  {"bn_bwd_cap", kBnBwdCap},
    {"row_reduce", kRowReduce},      {"c3_epilogue", kC3Epilogue},   {"c3_window_kb", kC3WindowKB},
    {"tg_ws", kTgWs},                {"tg_ps", kTgPs},               {"bn_fin_act", kBnFinAct},
    {"tg_split_k", kTgSplitK},
};

extern int g_tune[kTuneSlots];

}  // namespace dcp
