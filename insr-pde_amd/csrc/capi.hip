// capi.hip -- the C ABI of libinsr_hip.so (include/insr_siren.h): argument checks,
// kernel-variant selection, the partial reducer and the device-resident optimiser.
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "jet_common.hpp"
#include "optim.hpp"

namespace insr {

int streams_for(int din, int mode) {
  if (mode == INSR_MODE_VALUE) return 1;
  if (mode == INSR_MODE_GRAD) return 1 + din;
  if (mode == INSR_MODE_LAP) return 2 + din;
  return -1;
}

int nt_for(int width) {
  if (width == 32) return 2;
  if (width == 64) return 4;
  if (width == 128) return 8;
  if (width == 256) return 16;  // tile-split kernels only
  return -1;
}

// Per-call knobs, decoded from the `mode` argument of every call (include/insr_siren.h:
// INSR_JET_POLICY, INSR_JET_BWD_F16, INSR_JET_TILES, INSR_MODE_WIDE128; the precisions are
// INSR_JET_PREC / INSR_JET_BPREC).  The library holds no mutable process-wide configuration and
// reads no environment: two calls on distinct streams (threads) with different knobs never see
// each other's, and a field left 0 takes the measured default below.
constexpr int kMinBlocksDefault = 256;
constexpr int kBwdF16Default = INSR_BWD_F16_DW | INSR_BWD_F16_PROP | INSR_BWD_F16_FUSED;  // profiles/r03/bwd_f16_ab
struct Knobs {
  int policy;    // backward path: 0 auto, 1 fused, 2 two-kernel, 3 resident dW, 4 recompute,
                 // 5 resident dW with f16x3 products (the saved-stream jet_fb variant)
  int f16;       // INSR_BWD_F16_* mask: x6 backward products on the fp16 matrix cores
  int wide_min;  // smallest width of the two-kernel backward (128 or 256)
  int tiles[3];  // forced forward T, forced backward T (0 = auto), minimum block count
};
static int tiles_of_code(int c) { return c == 3 ? 4 : c; }  // 0 auto, 1, 2, 4
static int min_blocks_of_code(int c) {
  static constexpr int v[4] = {kMinBlocksDefault, 512, 128, 1024};
  return v[c & 3];
}
Knobs knobs_of(int mode) {
  Knobs k;
  const int pol = (mode >> INSR_MODE_POLICY_SHIFT) & 7, f = (mode >> INSR_MODE_F16_SHIFT) & 0xF;
  const int t = (mode >> INSR_MODE_TILES_SHIFT) & 0x3F;
  k.policy = pol ? pol - 1 : 0;
  k.f16 = f ? f - 1 : kBwdF16Default;
  k.wide_min = (mode & INSR_MODE_WIDE128) ? 128 : 256;
  k.tiles[0] = tiles_of_code(t & 3);
  k.tiles[1] = tiles_of_code((t >> 2) & 3);
  k.tiles[2] = min_blocks_of_code(t >> 4);
  return k;
}
static bool knobs_ok(int mode) {
  const int pol = (mode >> INSR_MODE_POLICY_SHIFT) & 7, f = (mode >> INSR_MODE_F16_SHIFT) & 0xF;
  return pol <= 6 && f <= 8;
}

// The recompute backward (jet_fb.hpp: forward + reverse jet per tile in one persistent launch, no
// saved streams) serves W = 128 nets of 4 hidden layers at the fp32-level backward precision
// (its products are f16x3 with per-tile scales).  The decision must not depend on n (the forward
// of the same call skips its saved streams).  Forced by policy 4 only: measured 196 us at 16,708
// Laplacian points vs 172 us for the two-kernel backward (kbench r4e, profiles/r04/) --
// VALU / barrier-latency bound, see DESIGN.md.
bool use_fb(int S, int NT, bool lap, int nq, int L, const Knobs& k) {
  if (NT != 8 || nq != 3 || !fb_supported(S, lap, L)) return false;
  return k.policy == 4;
}

// The resident-dW backward (jet_x6r.hpp) serves W = 128 nets of 4 hidden layers (the fluid
// nets; compiled for that depth only) at x6 precision: value, 2-d gradient and 2-d Laplacian
// jets.  Auto policy (8-wave blocks; kbench r3c, profiles/r03/kbench_policies.jsonl, backward
// into .grad incl. sums): Laplacian jets from 32,768 points (33,092: 325 vs 340 us two-kernel;
// 65,536: 544 vs 632), value jets from 49,152 (65,536: 171-177 vs 224-234; 33,092 equal;
// 16,708: 80 vs 64-69 fused -- below ~8 tiles per CU the 64 MB of per-CU dW partials dominate).
bool resident_ok(int S, int NT, bool lap, int nq, int L) {
  if (NT != 8 || nq != 3) return false;
  if (L == 5) return S == 3 && !lap;  // (the jet_fb.hpp saved-stream sweep only: jet_x6r is compiled for L = 4)
  if (L != 4) return false;
  return (S == 1 && !lap) || (S == 3 && !lap) || (S == 4 && lap);
}
// Round 3: with the two-kernel path's products on the fp16 matrix cores (INSR_BWD_F16_DW | PROP;
// the resident kernel stays bf16x6) the two-kernel Laplacian backward wins at the fluid2DtlgnM batch
// (66,844 points: 553-561 vs 590-601 us; value jets tie at 199-205, profiles/r03/final_r3o/
// kbench_policy_M.jsonl), so the auto policy keeps the resident kernel for value jets only then.
bool use_resident_f16(long n, int S, int NT, bool lap, int nq, int L, const Knobs& k);
bool use_resident(long n, int S, int NT, bool lap, int nq, int L, const Knobs& k) {
  if (!resident_ok(S, NT, lap, nq, L)) return false;
  if (L == 5) return use_resident_f16(n, S, NT, lap, nq, L, k);  // no jet_x6r instantiation at this depth
  if (k.policy == 3 || k.policy == 5) return true;
  if (k.policy != 0) return false;
  if (use_resident_f16(n, S, NT, lap, nq, L, k)) return true;
  const bool f16w = (k.f16 & (INSR_BWD_F16_DW | INSR_BWD_F16_PROP)) == (INSR_BWD_F16_DW | INSR_BWD_F16_PROP);
  return lap ? (!f16w && n >= 32768) : (S == 1 && n >= 49152);
}

// Which kernel serves the resident path: the saved-stream variant of the recompute kernel (jet_fb.hpp
// SAVED: the reverse sweep on the forward's saved streams, f16x3 products with per-tile scales; the
// INSR_BWD_F16_FUSED bit of the call's mask) or jet_x6r.hpp (bf16x6 products).  Policy 5 forces the
// former.  Auto: 2-d Laplacian jets from 4,096 points -- backward into .grad incl. sums (kbench r4j,
// profiles/r04/kbench_resident_f16.jsonl): 16,708 points 142 vs 166 us two-kernel, 33,092 239 vs
// 296-301, 66,844 428 vs 577-582; value jets lose at every size (S = 1: 16-point tiles, 90 vs 57 fused
// at 16,708), so they keep their paths.  Round 4, with both backwards' sums in the Adam launch: from
// 4,096 points (the fluid2DtlgnM 8-way shard step, 8,192 + 163 points: 0.331-0.332 vs 0.345-0.347 ms
// with the two-kernel path, profiles/r04/ab_fb_shard/).
bool use_resident_f16(long n, int S, int NT, bool lap, int nq, int L, const Knobs& k) {
  if (NT != 8 || nq != 3 || !fb_saved_supported(S, lap, L)) return false;
  if (k.policy == 5) return true;
  if (k.policy != 0 || !(k.f16 & INSR_BWD_F16_FUSED)) return false;
  // round 6: also the 5-layer 2-d gradient jet (the el2D deformation net's Jacobian) from 4,096 points
  return (lap && S == 4 && n >= 4096) || (!lap && S == 3 && L == 5 && n >= 4096);
}

// Matrix-core precision of the tile-split kernels (a call's INSR_JET_PREC(p) / INSR_JET_BPREC(p);
// base.MLP(precision=...) sets them per network), else the defaults:
//   INSR_PREC_F32     v_mfma_f32_16x16x4_f32 (jet_split.hpp)
//   INSR_PREC_BF16X6  split-bf16, 6 products (jet_x6.hpp, NQ = 3): fp32-level accuracy (default backward)
//   INSR_PREC_F16X3   fp16 two terms, 3 products (NQ = 4): fp32-level accuracy, forward only (default forward)
//   INSR_PREC_BF16X3  split-bf16, 3 products (NQ = 2)
//   INSR_PREC_BF16    bf16 operands, fp32 accumulation (NQ = 1)
// Default forward f16x3 (fields <= 4.2e-6, gradients <= 5.1e-6 vs the oracle like x6's 3.5e-6 /
// 5.1e-6, profiles/r03/prec_f16x3.jsonl; forward jets 15-30 % faster, profiles/r03/f16x3_ab) and the
// split-bf16 x6 backward (same accuracy as fp32 MFMA, measured faster: profiles/r01/kbench_x6.jsonl)
constexpr int kPrecDefault[2] = {INSR_PREC_F16X3, INSR_PREC_BF16X6};

static bool prec_ok(int p) { return p >= INSR_PREC_F32 && p <= INSR_PREC_F16X3; }

// precision of a call (direction bwd): the mode's backward override (bwd), else its
// override, else the default
int call_prec(int mode, int bwd) {
  const int pb = (mode >> INSR_MODE_BPREC_SHIFT) & 0xF;
  const int po = (mode >> INSR_MODE_PREC_SHIFT) & 0xF;
  const int p = (bwd && pb) ? pb - 1 : (po ? po - 1 : kPrecDefault[bwd ? 1 : 0]);
  // f16x3 is a forward precision: its backward runs the fp32-level split-bf16 kernels
  return (bwd && p == INSR_PREC_F16X3) ? INSR_PREC_BF16X6 : p;
}

// bf16 terms per operand of a precision (0: the exact-fp32 tile-split kernels)
int nq_of(int prec) {
  return prec == INSR_PREC_F16X3 ? 4 : prec == INSR_PREC_BF16X6 ? 3 : prec == INSR_PREC_BF16X3 ? 2
                                                                     : prec == INSR_PREC_BF16 ? 1 : 0;
}

// Backward through the two-kernel path (jet_x6w.hpp: propagation kernel + split-K dW GEMM)
// for the split-bf16 precisions at widths >= wide_min (default 256; INSR_MODE_WIDE128 for A/B
// studies) and, at width 128, for Laplacian jets of >= 8192 points and 3-4
// stream gradient jets of >= 32768 points.  Measured (profiles/r02/kbench_wide_vs_fused.jsonl,
// backward into .grad incl. reductions): LAP 16384 points 244 -> 182 us, LAP 65536 813 -> 698,
// GRAD (S = 3) 65536 595 -> 548; GRAD 16384 140 vs 144 and every value jet stay fused.
bool use_wide(long n, int S, int NT, bool lap, int nq, const Knobs& k) {
  if (NT < 8 || nq == 0) return false;
  if (k.policy == 2) return true;
  if (k.policy == 1 && NT == 8) return false;
  if (16 * NT >= k.wide_min) return true;
  if (NT != 8 || k.wide_min > 256) return false;
  // with the pre-split weight planes (kbench r2s31, profiles/r02/wide_vs_fused_wsplit.jsonl):
  // Laplacian and 2-d gradient jets from 8,192 points (gradient 16,708: 143 vs 175 us fused),
  // value jets from ~24K points: round 3, f16x3 products on both paths (kbench r3aa, backward
  // into .grad incl. sums, profiles/r03/kbench_value_routing.jsonl): 16,708 fused 54.4-56.1 vs
  // two-kernel 60.9-62.4 us; 33,092 fused 101.7-103.7 vs two-kernel 93.4-95.3 (>= 49,152: resident)
  if (lap || S >= 3) return n >= 8192;
  return S == 1 && n >= 24576;
}

static int cu_count() { return device_cus(); }

// per-precision dispatch (nq = 0: exact fp32)
static int fwd_q(int nq, int NT, int S, bool lap, int T, const float* x, int N, int din, int dout, int L,
                 const float* prm, float* y, float* dy, float* lp, float* act, int nbal, hipStream_t st) {
  switch (nq) {
    case 4: return dispatch_fwd_q<4>(NT, S, lap, T, x, N, din, dout, L, prm, y, dy, lp, act, nbal, st);
    case 3: return dispatch_fwd_q<3>(NT, S, lap, T, x, N, din, dout, L, prm, y, dy, lp, act, nbal, st);
    case 2: return dispatch_fwd_q<2>(NT, S, lap, T, x, N, din, dout, L, prm, y, dy, lp, act, nbal, st);
    case 1: return dispatch_fwd_q<1>(NT, S, lap, T, x, N, din, dout, L, prm, y, dy, lp, act, nbal, st);
    default: return dispatch_fwd_split(NT, S, lap, T, x, N, din, dout, L, prm, y, dy, lp, act, st);
  }
}
// the kernel precision of a fused tile-split backward at precision nq: the x6 backward's products on
// the fp16 matrix cores under INSR_BWD_F16_FUSED (jet_h_bwd.hip)
static int fused_bwd_nq(int nq, const Knobs& k) { return (nq == 3 && (k.f16 & INSR_BWD_F16_FUSED)) ? 4 : nq; }

// J == NULL: occupancy query; the exact-fp32 kernel takes one job per launch
static int bwd_q(int nq, int NT, int S, bool lap, int T, const BwdJobsX6* J, int din, int dout, int L,
                 const float* prm, float* part, long P, hipStream_t st) {
  switch (nq) {
    case 4: return dispatch_bwd_q<4>(NT, S, lap, T, J, din, dout, L, prm, part, P, st);
    case 3: return dispatch_bwd_q<3>(NT, S, lap, T, J, din, dout, L, prm, part, P, st);
    case 2: return dispatch_bwd_q<2>(NT, S, lap, T, J, din, dout, L, prm, part, P, st);
    case 1: return dispatch_bwd_q<1>(NT, S, lap, T, J, din, dout, L, prm, part, P, st);
    default:
      if (!J)
        return dispatch_bwd_split(NT, S, lap, T, nullptr, -1, 0, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr,
                                  nullptr, 0, nullptr);
      if (J->njobs != 1) return INSR_EINVAL;
      return dispatch_bwd_split(NT, S, lap, T, J->x[0], J->n[0], din, dout, L, prm, J->act[0], J->gy[0], J->gdy[0],
                                J->glap[0], part, P, st);
  }
}

// resident blocks per CU of a tile-split kernel instantiation (launchers answer N < 0)
static int occupancy(int bwd, int nq, int NT, int S, bool lap, int T) {
  static std::mutex mu;  // calls from several host threads (one per stream) share the cache
  static std::map<int, int> cache;
  const int key = (((((bwd * 8 + nq) * 32 + NT) * 8 + S) * 2 + (lap ? 1 : 0)) * 8) + T;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  const int r = bwd ? bwd_q(nq, NT, S, lap, T, nullptr, 0, 0, 0, nullptr, nullptr, 0, nullptr)
                    : fwd_q(nq, NT, S, lap, T, nullptr, -1, 0, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                            nullptr);
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = r;
  return r;
}

// Tiles per tile-split block.  The largest T in {1, 2, 4} whose LDS fits a CU,
// lowered while the grid would have fewer than the call's minimum block count (small batches
// want many short blocks, large ones fewer blocks that share W fetches, barriers
// and partial rows).  A call may force T per direction (INSR_JET_TILES: A/B studies).
int split_tiles(int bwd, int NT, int S, long n, bool lap, int nq, const Knobs& k) {
  const bool x6 = nq > 0;
  // LDS per tile: fp32 planes [S][16][W+8] (+ backward h planes [S][16][W]); split-bf16
  // forward: NQ bf16 planes [S][NQ][16][W+8]; backward: one stream group of bf16 Z + H planes
  // (the kernel picks the group size that fits, jet_x6.hpp x6_bwd_sg)
  const int np = nq == 4 ? 2 : nq;  // LDS planes per value (f16x3: two fp16 terms)
  const size_t plane = x6 && !bwd ? (size_t)S * np * 16 * (16 * NT + 8) * 2
                       : x6       ? (size_t)(nq * 16 * (16 * NT + 8) + 32 + nq * 16 * 16 * NT) * 2
                                  : (size_t)S * 16 * ((16 * NT + 8) + (bwd ? 16 * NT : 0)) * sizeof(float);
  // width 256: fp32 kernels one tile (register budget of 8 waves x 2 row tiles); the x6
  // forward T x S <= 4 (its a[T][2][S] accumulators next to the 8 split W fragments);
  // backward T = 4 only for value jets (register budget of the derivative streams)
  int T = NT > 8 ? ((x6 && !bwd) ? (S == 1 ? 4 : (S == 2 ? 2 : 1)) : 1) : ((bwd && S > 1) ? 2 : 4);
  while (T > 1 && (size_t)T * plane > 163840) T >>= 1;
  const int forced = k.tiles[bwd ? 1 : 0];
  if (forced > 0) {  // the largest feasible T not above the forced one
    while (T > forced) T >>= 1;
    return T;
  }
  // x6 forward of 4-stream jets (Laplacian, 3-d gradient) at W <= 128: T = 1 measured faster
  // than the LDS-capped T = 2 (16384 points: 66.6 vs 71.5 us, kbench s32)
  if (x6 && !bwd && S >= 4 && NT <= 8) T = 1;
  const long tiles = (n + 15) / 16;
  // x6 forward at W = 128 with the pre-split weight planes (62-90 VGPRs: 2-4 blocks per CU),
  // measured per tile count (kbench r2s29, profiles/r02/tiles_after_wsplit.jsonl): value jets
  // T = 2 up to ~40K points (16,708: 26.4 vs 29.8 us at T = 4; 33,092: 41.5 vs 47.2), T = 4
  // above (65,536: 60.2 vs 64.9); 2-4 stream jets T = 1 (16,708: 48.2 vs 58.3 at T = 2)
  if (x6 && !bwd && NT == 8) {
    if (S > 1) return 1;
    return tiles <= 512 ? 1 : (tiles <= 2600 ? 2 : 4);
  }
  while (T > 1 && (tiles + T - 1) / T < k.tiles[2]) T >>= 1;
  // occupancy-aware: a T whose last round of blocks (resident blocks per CU x CUs) is
  // nearly empty loses to a smaller T that packs the CUs, e.g. the x6 gradient forward at
  // 20,000 points: T = 4 -> 313 one-per-CU blocks = 2 rounds (97 us) vs T = 1 -> 1250
  // two-per-CU blocks (68 us; profiles/r01/kbench_tiles_s44.jsonl).  Cost = rounds x T.
  if (T > 1) {
    const int cus = cu_count();
    auto cost = [&](int t) -> double {
      const int o = occupancy(bwd, nq, NT, S, lap, t);
      if (o <= 0) return 1e30;
      const long nb = (tiles + t - 1) / t, per = (long)o * cus;
      return (double)((nb + per - 1) / per) * t;
    };
    const double c0 = cost(T);
    for (int t = T >> 1; t >= 1; t >>= 1)
      if (c0 > 2.2 * cost(t)) {
        T = t;
        break;
      }
  }
  return T;
}

// Balanced launch shape: T tiles per block from split_tiles; if the batch overflows the last
// round of resident blocks by a little (16384 interior + 324 band points = 1045 tiles on
// 256 one-block CUs: 262 blocks, 2 rounds), blocks of up to T + 1 tiles (T = 4 -> 5 for
// value jets, 2 -> 3 for 2-3 stream jets) spread the tiles evenly over fewer blocks when that
// saves a round.  nbal = the block count (0: plain T-tile blocks).
struct LaunchShape {
  int T, nbal;
};
LaunchShape launch_shape(int bwd, int nq, int NT, int S, bool lap, long n, const Knobs& k) {
  LaunchShape sh{split_tiles(bwd, NT, S, n, lap, nq, k), 0};
  if (nq == 0 || NT > 8 || lap || k.tiles[bwd ? 1 : 0] > 0) return sh;  // exact fp32 / forced T: plain
  if (bwd && S == 1 && NT == 8 && k.tiles[2] == kMinBlocksDefault) {
    // x6 value backward at W = 128 (unless an A/B study set its own minimum block count): every block writes one full partial-gradient row (P floats)
    // that reduce_partials re-reads, so below ~5 tiles per CU the block count, not the CU fill,
    // sets the time.  About half as many blocks as CUs wins (kbench r3d, fluid_vel, backward +
    // reduction): 4,178 points 131 x T = 2 35.4 us vs 262 x T = 1 58.5; 8,354 points 131 x T = 4
    // 45.6 vs 262 x T = 2 66.4; 16,708 points 209 x 5 (balanced) 63.1 vs 262 x T = 4 86.8.
    const long tiles = (n + 15) / 16, half = (cu_count() + 1) / 2, lim = half + half / 20;
    if (tiles <= lim) return LaunchShape{1, 0};
    if (tiles <= 2 * lim) return LaunchShape{2, 0};
    if (tiles <= 4 * lim) return LaunchShape{4, 0};
    if (tiles <= 5L * cu_count()) return LaunchShape{5, (int)((tiles + 4) / 5)};
  }
  // backward: value jets only (the 3-tile gradient backward spills: 280 B of scratch per lane)
  const int T1 = sh.T == 4 && S == 1 ? 5 : (!bwd && sh.T == 2 && (S == 2 || S == 3) ? 3 : 0);
  if (!T1) return sh;
  const int cus = cu_count();
  const int o = occupancy(bwd, nq, NT, S, lap, sh.T), o1 = occupancy(bwd, nq, NT, S, lap, T1);
  if (o <= 0 || o1 <= 0) return sh;
  const long tiles = (n + 15) / 16;
  const long nb = (tiles + sh.T - 1) / sh.T, slots = (long)o * cus, slots1 = (long)o1 * cus;
  const long rounds = (nb + slots - 1) / slots;
  const long nb1 = (tiles + T1 - 1) / T1, rounds1 = (nb1 + slots1 - 1) / slots1;
  if (rounds1 >= rounds) return sh;
  long nbal = rounds1 * slots1;  // as many blocks as the rounds hold (fewest tiles per block) ...
  if (nbal > nb) nbal = nb;      // ... but never below the plain shape's tiles per block
  if (nbal < nb1) nbal = nb1;
  sh.T = T1;
  sh.nbal = (int)nbal;
  return sh;
}

constexpr int kRedWaves = 8;
__global__ __launch_bounds__(64 * kRedWaves) void reduce_partials_kernel(const float* __restrict__ part, int nb,
                                                                          long count, float* __restrict__ grad,
                                                                          int accumulate) {
  // block: 64 columns (lanes) x kRedWaves row slices; fixed summation order
  __shared__ float red[kRedWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long i = (long)blockIdx.x * 64 + lane;
  float acc = 0.f;
  if (i < count) {
    int b = w;
    for (; b + 3 * kRedWaves < nb; b += 4 * kRedWaves) {
      const float a0 = part[(long)b * count + i];
      const float a1 = part[(long)(b + kRedWaves) * count + i];
      const float a2 = part[(long)(b + 2 * kRedWaves) * count + i];
      const float a3 = part[(long)(b + 3 * kRedWaves) * count + i];
      acc += a0;
      acc += a1;
      acc += a2;
      acc += a3;
    }
    for (; b < nb; b += kRedWaves) acc += part[(long)b * count + i];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && i < count) {
    float s = accumulate ? grad[i] : 0.f;
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kRedWaves; ++k) t += red[k][lane];
    grad[i] = s + t;
  }
}

// Partial rows padded to a multiple of 4 floats (insr_jet_partial_stride): 16-B aligned
// rows, so the reduction streams them with 16-B loads (1 KiB per wave-instruction) and
// 8 rows in flight per thread.  Fixed summation order as reduce_partials_kernel.
constexpr int kRed4Waves = 8, kRed4Unroll = 16;  // rows in flight per thread (predicated tail)
__global__ __launch_bounds__(64 * kRed4Waves) void reduce_partials4_kernel(const float* __restrict__ part, int nb,
                                                                            long count, long stride,
                                                                            float* __restrict__ grad, int accumulate,
                                                                            LossFin fin = LossFin{}) {
  __shared__ floatx4 red[kRed4Waves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // fin.nloss > 0: the grid's extra last block (no columns of its own) finishes the loss values
  if (fin.nloss && blockIdx.x == gridDim.x - 1 && w == 0) loss_finalize(fin);
  const long q = (long)blockIdx.x * 64 + lane;  // column quad
  floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
  if (4 * q < count) {
    const floatx4* col = reinterpret_cast<const floatx4*>(part) + q;
    const long rs = stride / 4;
    // rows w, w + 8, ... in order (the fixed summation order); a batch's rows past nb add zeros
    for (int b = w; b < nb; b += kRed4Unroll * kRed4Waves) {
      floatx4 v[kRed4Unroll];
#pragma unroll
      for (int u = 0; u < kRed4Unroll; ++u) {
        const int r = b + u * kRed4Waves;
        v[u] = r < nb ? col[(long)r * rs] : floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < kRed4Unroll; ++u) acc += v[u];
    }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && 4 * q < count) {
    floatx4 t = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < kRed4Waves; ++k) t += red[k][lane];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long i = 4 * q + r;
      if (i < count) grad[i] = accumulate ? grad[i] + t[r] : t[r];
    }
  }
}

// First level of a two-level reduction for many rows: block (x, y) sums rows
// [y R, (y + 1) R) of its 256 columns and writes the sum into row y R (in place: those
// rows are read only by this block, before the write); the second level is
// reduce_partials4_kernel over the slice rows (row stride R * stride).
__global__ __launch_bounds__(64 * kRed4Waves) void reduce_slices4_kernel(float* __restrict__ part, int nb, int R,
                                                                          long count, long stride) {
  __shared__ floatx4 red[kRed4Waves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long q = (long)blockIdx.x * 64 + lane;
  const int b0 = blockIdx.y * R, b1 = min(nb, b0 + R);
  floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
  floatx4* col = reinterpret_cast<floatx4*>(part) + q;
  const long rs = stride / 4;
  if (4 * q < count) {
    for (int b = b0 + w; b < b1; b += kRed4Unroll * kRed4Waves) {
      floatx4 v[kRed4Unroll];
#pragma unroll
      for (int u = 0; u < kRed4Unroll; ++u) {
        const int r = b + u * kRed4Waves;
        v[u] = r < b1 ? col[(long)r * rs] : floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < kRed4Unroll; ++u) acc += v[u];
    }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && 4 * q < count && b0 < nb) {
    floatx4 t = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < kRed4Waves; ++k) t += red[k][lane];
    col[(long)b0 * rs] = t;  // 16-B store; the row's padding columns are never summed
  }
}

__global__ void adam_prepare_kernel(float* st, float b1, float b2) {
  // legacy explicit prepare: t += 1 and refresh the bias-corrected scalars
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const double t = (double)st[INSR_OPT_STEP] + 1.0;
    st[INSR_OPT_STEP] = (float)t;
    st[INSR_OPT_STEPSIZE] = (float)((double)st[INSR_OPT_LR] / (1.0 - pow((double)b1, t)));
    st[INSR_OPT_BC2SQRT] = (float)sqrt(1.0 - pow((double)b2, t));
  }
}

__global__ void plateau_kernel(float* st, const float* loss, int patience, int advance_step) {
  if (threadIdx.x == 0 && blockIdx.x == 0) plateau_update(st, loss, patience, advance_step);
}

struct AdamList {
  float* p[INSR_ADAM_MAX_TENSORS];
  const float* g[INSR_ADAM_MAX_TENSORS];
  float* m[INSR_ADAM_MAX_TENSORS];
  float* v[INSR_ADAM_MAX_TENSORS];
  long n[INSR_ADAM_MAX_TENSORS];
  long start[INSR_ADAM_MAX_TENSORS + 1];  // prefix sums of n
  int shape[INSR_ADAM_MAX_TENSORS][4];    // SIREN (d_in, d_out, L, W) of a flat buffer with weight planes, else 0s
  const float* loss;                      // != NULL: the last block runs the plateau step on it
  int patience;
  int count;
};

__global__ void adam_multi_kernel(AdamList L, float* __restrict__ st, float b1, float b2, float eps,
                                  int step_offset) {
  __shared__ float sc[2];
  if (threadIdx.x == 0) {
    const double t = (double)st[INSR_OPT_STEP] + (double)step_offset;
    double p1, p2;
    powi2_d((double)b1, (double)b2, (unsigned)t, p1, p2);
    sc[0] = (float)((double)st[INSR_OPT_LR] / (1.0 - p1));
    sc[1] = (float)sqrt(1.0 - p2);
  }
  __syncthreads();
  const float step_size = sc[0], bc2s = sc[1];
  const float w1 = (float)(1.0 - (double)b1);
  const float w2 = (float)(1.0 - (double)b2);
  const long total = L.start[L.count];
  for (long gi = (long)blockIdx.x * blockDim.x + threadIdx.x; gi < total; gi += (long)gridDim.x * blockDim.x) {
    int k = 0;
    while (k + 1 < L.count && gi >= L.start[k + 1]) ++k;
    const long i = gi - L.start[k];
    float mi, vi;
    const float pn = adam_elem(L.g[k][i], L.m[k][i], L.v[k][i], L.p[k][i], step_size, bc2s, w1, w2, b2, eps, mi, vi);
    L.m[k][i] = mi;
    L.v[k][i] = vi;
    L.p[k][i] = pn;
    if (L.shape[k][2] > 0) adam_wsplit(L.p[k], L.shape[k], i, pn);
  }
  // fused scheduler step: every block read lr / t above before it takes a ticket (relaxed ticket,
  // no release/acquire: the last block only reads the loss -- written by an earlier launch -- and
  // st, which no other block writes; the plain loads of lr / t above completed before each block's
  // barrier)
  if (L.loss) plateau_after_blocks(st, L.loss, L.patience, blockIdx.x, gridDim.x);
}

// The partial-row sums of a backward (reduce_partials4_kernel: the same rows per wave in the same
// order, the same cross-wave combine -- bit-identical gradients) with the Adam update of those
// elements as its epilogue, and the plateau step after the last block: one launch where the fused
// backward path took two (sums, then adam_multi_kernel).  grad receives the gradient as well (the
// flat .grad stays what torch would hold after backward()).  t = st[STEP] + 1, as the fused
// Adam + plateau launch; loss == NULL: Adam only (the caller advances t).
__global__ __launch_bounds__(64 * kRed4Waves) void reduce_adam_kernel(const float* __restrict__ part, int nb,
                                                                      long count, long stride,
                                                                      float* __restrict__ grad, int accumulate,
                                                                      float* __restrict__ p, float* __restrict__ m,
                                                                      float* __restrict__ v, int4 shp,
                                                                      float* __restrict__ st, float b1, float b2,
                                                                      float eps, const float* loss, int patience,
                                                                      LossFin fin = LossFin{}) {
  __shared__ floatx4 red[kRed4Waves][64];
  __shared__ float sc[2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // fin.nloss > 0: the grid's extra last block (no elements of its own) finishes the loss values
  // before its plateau ticket -- the plateau's last block then reads them (loss_finalize hand-off)
  if (fin.nloss && blockIdx.x == gridDim.x - 1 && w == 0) loss_finalize(fin);
  if (threadIdx.x == 0) {
    const double t = (double)st[INSR_OPT_STEP] + 1.0;
    double p1, p2;
    powi2_d((double)b1, (double)b2, (unsigned)t, p1, p2);
    sc[0] = (float)((double)st[INSR_OPT_LR] / (1.0 - p1));
    sc[1] = (float)sqrt(1.0 - p2);
  }
  // the Adam epilogue's element (threads 0..255: element blockIdx.x * 256 + threadIdx.x): its state
  // is loaded before the sums, under their latency
  const long ie = (long)blockIdx.x * 256 + threadIdx.x;
  const bool mine = threadIdx.x < 256 && ie < count;
  float g0 = 0.f, m0 = 0.f, v0 = 0.f, p0 = 0.f;
  if (mine) {
    m0 = m[ie];
    v0 = v[ie];
    p0 = p[ie];
    if (accumulate) g0 = grad[ie];
  }
  const long q = (long)blockIdx.x * 64 + lane;  // column quad
  floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
  if (4 * q < count) {
    const floatx4* col = reinterpret_cast<const floatx4*>(part) + q;
    const long rs = stride / 4;
    for (int b = w; b < nb; b += kRed4Unroll * kRed4Waves) {
      floatx4 vv[kRed4Unroll];
#pragma unroll
      for (int u = 0; u < kRed4Unroll; ++u) {
        const int r = b + u * kRed4Waves;
        vv[u] = r < nb ? col[(long)r * rs] : floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < kRed4Unroll; ++u) acc += vv[u];
    }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0) {  // the cross-wave sums in reduce_partials4_kernel's order, back into red[0]
    floatx4 tt = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < kRed4Waves; ++k) tt += red[k][lane];
    red[0][lane] = tt;
  }
  __syncthreads();
  if (mine) {  // torch's op order, as adam_multi_kernel
    const float tsum = reinterpret_cast<const float*>(&red[0][0])[threadIdx.x];
    const float g = accumulate ? g0 + tsum : tsum;
    grad[ie] = g;
    const float step_size = sc[0], bc2s = sc[1];
    const float w1 = (float)(1.0 - (double)b1);
    const float w2 = (float)(1.0 - (double)b2);
    float mi, vi;
    const float pn = adam_elem(g, m0, v0, p0, step_size, bc2s, w1, w2, b2, eps, mi, vi);
    m[ie] = mi;
    v[ie] = vi;
    p[ie] = pn;
    if (shp.z > 0) {
      const int sh4[4] = {shp.x, shp.y, shp.z, shp.w};
      adam_wsplit(p, sh4, ie, pn);
    }
  }
  if (loss) plateau_after_blocks(st, loss, patience, blockIdx.x, gridDim.x);
}

bool shape_ok(int din, int dout, int L, int width, int mode) {
  if (din < 1 || din > 3 || dout < 1 || dout > 3 || L < 0 || L > 64) return false;
  if (nt_for(width) < 0) return false;
  if (mode & ~(INSR_MODE_MASK | (0xF << INSR_MODE_PREC_SHIFT) | (0xF << INSR_MODE_BPREC_SHIFT) | INSR_MODE_WSPLIT |
               INSR_MODE_WIDE128 | (7 << INSR_MODE_POLICY_SHIFT) | (0xF << INSR_MODE_F16_SHIFT) |
               (0x3F << INSR_MODE_TILES_SHIFT)))
    return false;
  if (!knobs_ok(mode)) return false;
  const int po = (mode >> INSR_MODE_PREC_SHIFT) & 0xF, pb = (mode >> INSR_MODE_BPREC_SHIFT) & 0xF;
  if ((po && !prec_ok(po - 1)) || (pb && !prec_ok(pb - 1))) return false;
  const int jm = mode & INSR_MODE_MASK;
  const int S = streams_for(din, jm);
  if (S < 1 || S > 5) return false;  // the Laplacian jet of a 3-d input carries 5 streams
  // ... whose exact-fp32 backward at width 256 does not fit a CU's LDS (5 x 16 x 520 floats)
  if (S == 5 && nt_for(width) == 16 && (nq_of(call_prec(mode, 0)) == 0 || nq_of(call_prec(mode, 1)) == 0)) return false;
  return true;
}

// one jet call's configuration: jet mode, streams, row tiles, bf16 terms per direction, knobs
struct JetCall {
  int jm, S, NT, nqf, nqb;
  bool lap;
  Knobs k;
  JetCall(int din, int W, int mode)
      : jm(mode & INSR_MODE_MASK),
        S(streams_for(din, mode & INSR_MODE_MASK)),
        NT(nt_for(W)),
        nqf(nq_of(call_prec(mode, 0))),
        nqb(nq_of(call_prec(mode, 1))),
        lap((mode & INSR_MODE_MASK) == INSR_MODE_LAP),
        k(knobs_of(mode)) {}
  bool ok() const { return S > 0 && NT > 0; }
  // width 256 has no fused split-bf16 backward: the two-kernel path serves it
  bool wide(long n) const { return use_wide(n, S, NT, lap, nqb, k); }
  bool resident(long n, int L) const { return use_resident(n, S, NT, lap, nqb, L, k); }
  bool recompute(int L) const { return use_fb(S, NT, lap, nqb, L, k); }
  bool resident_f16(long n, int L) const { return resident(n, L) && use_resident_f16(n, S, NT, lap, nqb, L, k); }
  // 0: fused tile-split + partial rows (insr_siren_jet_bwd), 1: two-kernel, 2: resident dW,
  // 3: recompute (no saved streams)
  int path(long n, int L) const { return recompute(L) ? 3 : (resident(n, L) ? 2 : (wide(n) ? 1 : 0)); }
};

}  // namespace insr

using namespace insr;

extern "C" {

int insr_version(void) { return 300; }

long insr_siren_param_count(int din, int dout, int L, int W) {
  return (long)W * din + W + (long)L * ((long)W * W + W) + (long)dout * W + dout;
}

long insr_jet_partial_stride(int din, int dout, int L, int W) {
  return (insr_siren_param_count(din, dout, L, W) + 3) & ~3L;  // 16-B aligned rows
}

// ---- pre-split weight planes --------------------------------------------------------------
long insr_siren_wsplit_offset(int din, int dout, int L, int W) {
  if (!shape_ok(din, dout, L, W, 0)) return INSR_EINVAL;
  return wsplit_offset(din, dout, L, W);
}
long insr_siren_wsplit_floats(int L, int W) {
  if (L < 0 || nt_for(W) < 0) return INSR_EINVAL;
  return wsplit_total_floats(L, W);
}
int insr_siren_wsplit(float* params, int din, int dout, int L, int W, void* stream) {
  if (!params || !shape_ok(din, dout, L, W, 0)) return INSR_EINVAL;
  return wsplit_launch(params, din, dout, L, W, params + wsplit_offset(din, dout, L, W), (hipStream_t)stream);
}

// A call without INSR_MODE_WSPLIT whose kernels read weight planes: a per-(device, stream,
// slot) scratch [copy of the parameters | planes] is filled (one copy + one split launch) and
// used as the params buffer.  Allocation happens outside stream capture only.
namespace {
struct Scratch {
  void* ptr = nullptr;
  size_t bytes = 0;
};
std::mutex g_scratch_mu;
std::map<std::tuple<int, hipStream_t, int>, Scratch> g_scratch;
}  // namespace

static const float* with_planes(const float* params, int din, int dout, int L, int W, int mode, hipStream_t st,
                                int slot, int* rc) {
  *rc = 0;
  if ((mode & INSR_MODE_WSPLIT) || L < 1) return params;
  const long pc = insr_siren_param_count(din, dout, L, W);
  const size_t bytes = (size_t)(wsplit_offset(din, dout, L, W) + wsplit_total_floats(L, W)) * sizeof(float);
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  Scratch& e = g_scratch[std::make_tuple(dev, st, slot)];
  if (e.bytes < bytes) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cs);
    if (cs != hipStreamCaptureStatusNone) {
      *rc = INSR_ECAPTURE;
      return nullptr;
    }
    if (e.ptr) (void)hipFree(e.ptr);  // synchronous: no launch still reads the old copy
    e.ptr = nullptr;
    e.bytes = 0;
    if (hipMalloc(&e.ptr, bytes) != hipSuccess) {
      *rc = (int)hipErrorOutOfMemory;
      return nullptr;
    }
    e.bytes = bytes;
  }
  float* buf = static_cast<float*>(e.ptr);
  if ((*rc = (int)hipMemcpyAsync(buf, params, (size_t)pc * sizeof(float), hipMemcpyDeviceToDevice, st))) return nullptr;
  if ((*rc = wsplit_launch(buf, din, dout, L, W, buf + wsplit_offset(din, dout, L, W), st))) return nullptr;
  return buf;
}

int insr_siren_wsplit_status(const float* params, int din, int dout, int L, int W, void* stream) {
  if (!params || !shape_ok(din, dout, L, W, 0)) return INSR_EINVAL;
  if (L < 1) return 0;
  unsigned word = 0;
  if (const int rc = (int)hipStreamSynchronize((hipStream_t)stream)) return rc;
  if (const int rc = (int)hipMemcpy(&word, params + wsplit_status_offset(din, dout, L, W), sizeof(word),
                                    hipMemcpyDeviceToHost))
    return rc;
  return word ? INSR_ERANGE : 0;
}

int insr_siren_supported(int din, int dout, int L, int W, int mode) { return shape_ok(din, dout, L, W, mode) ? 1 : 0; }

long insr_jet_act_bytes(long n, int din, int L, int W, int mode) {
  const int S = streams_for(din, mode & INSR_MODE_MASK);
  if (S < 0 || n < 0) return INSR_EINVAL;
  const long tiles = act_tiles(n);
  return (long)(L + 1) * tiles * 16 * W * S * (long)sizeof(float);
}

long insr_jet_partial_bytes(long n, int din, int dout, int L, int W, int mode) {
  const int nb = insr_jet_partial_blocks(n, din, W, mode);
  if (nb < 0) return nb;
  return (long)nb * insr_jet_partial_stride(din, dout, L, W) * (long)sizeof(float);
}

int insr_siren_jet_fwd(const float* x, long n, int din, int dout, int L, int W, int mode, const float* params,
                       float* y, float* dy, float* lap, float* act, void* stream) {
  if (!shape_ok(din, dout, L, W, mode) || n < 0 || n > 0x7fffffffL) return INSR_EINVAL;
  if (n == 0) return 0;
  const JetCall c(din, W, mode);
  if (!x || !params || !y) return INSR_EINVAL;
  if (c.jm != INSR_MODE_VALUE && !dy) return INSR_EINVAL;
  if (c.lap && !lap) return INSR_EINVAL;
  const LaunchShape sh = launch_shape(0, c.nqf, c.NT, c.S, c.lap, n, c.k);
  int rc = 0;
  if (c.nqf > 0 && !(params = with_planes(params, din, dout, L, W, mode, (hipStream_t)stream, 0, &rc))) return rc;
  return fwd_q(c.nqf, c.NT, c.S, c.lap, sh.T, x, (int)n, din, dout, L, params, y, dy, lap, act, sh.nbal,
               (hipStream_t)stream);
}

int insr_siren_jet_fwd_multi(const InsrJetJob* jobs, int njobs, int din, int dout, int L, int W, int mode,
                             void* stream) {
  if (!jobs || njobs < 1 || njobs > INSR_MAX_FWD_JOBS || !shape_ok(din, dout, L, W, mode)) return INSR_EINVAL;
  const JetCall c(din, W, mode);
  long total = 0;
  int live = 0;
  for (int k = 0; k < njobs; ++k) {
    const InsrJetJob& j = jobs[k];
    if (j.n < 0 || j.n > 0x7fffffffL) return INSR_EINVAL;
    if (j.d_out < 0 || j.d_out > 3) return INSR_EINVAL;
    if (j.n == 0) continue;
    if (!j.x || !j.params || !j.y) return INSR_EINVAL;
    if (c.jm != INSR_MODE_VALUE && !j.dy) return INSR_EINVAL;
    if (c.lap && !j.lap) return INSR_EINVAL;
    total += j.n;
    ++live;
  }
  if (total > 0x7fffffffL) return INSR_EINVAL;
  if (live == 0) return 0;
  const int S = c.S, NT = c.NT;
  // one fused launch where the split-bf16 forward serves the combined batch; otherwise
  // (exact fp32, a Laplacian jet, a single job) the jobs launch one after another (the fused
  // kernel is compiled for widths 64 / 128 / 256)
  // W = 128 gradient jets fuse only while the batch fits one round of two 2-tile blocks per CU
  // (at 65,536 + 1,308 points the fused launch measured 4% slower per step than two launches)
  const bool grad128_big = NT == 8 && S == 3 && total > 2L * 2 * 16 * cu_count() + 4096;
  if (live > 1 && !c.lap && NT >= 4 && !grad128_big && c.nqf > 0) {
    // tiles per block from the combined batch; a job whose own batch would take fewer
    // (a boundary band) runs 1-tile blocks, placed first in the grid
    int T = split_tiles(0, NT, S, total, false, c.nqf, c.k);
    InsrJetJob pk[INSR_MAX_FWD_JOBS];
    int small[INSR_MAX_FWD_JOBS], nbal[INSR_MAX_FWD_JOBS];
    int m = 0;
    for (int k = 0; k < njobs; ++k)
      if (jobs[k].n > 0) {
        small[m] = split_tiles(0, NT, S, jobs[k].n, false, c.nqf, c.k) < T ? 1 : 0;
        nbal[m] = 0;
        pk[m] = jobs[k];
        int rc = 0;
        const int dk = jobs[k].d_out > 0 ? jobs[k].d_out : dout;
        if (!(pk[m].params = with_planes(jobs[k].params, din, dk, L, W, mode, (hipStream_t)stream, k, &rc))) return rc;
        ++m;
      }
    // value jets at T = 4 (two resident blocks per CU): when the jobs' blocks overflow a whole
    // round by a little (u_prev at 16384 points + u at 16384 + 324 band points: 518 blocks for
    // 512 slots), 5-tile blocks fit them in one round fewer
    if (T == 4 && S == 1 && NT <= 8) {
      const long slots = 2L * cu_count();
      long b4 = 0, b5 = 0;
      for (int k = 0; k < m; ++k) {
        const long tiles = (pk[k].n + 15) / 16;
        b4 += small[k] ? tiles : (tiles + 3) / 4;
        b5 += small[k] ? tiles : (tiles + 4) / 5;
      }
      if ((b5 + slots - 1) / slots < (b4 + slots - 1) / slots) T = 5;
    }
    hipStream_t st = (hipStream_t)stream;
    switch (c.nqf) {
      case 4: return dispatch_fwd_multi_q<4>(NT, S, false, T, pk, small, nbal, m, din, dout, L, st);
      case 3: return dispatch_fwd_multi_q<3>(NT, S, false, T, pk, small, nbal, m, din, dout, L, st);
      case 2: return dispatch_fwd_multi_q<2>(NT, S, false, T, pk, small, nbal, m, din, dout, L, st);
      default: return dispatch_fwd_multi_q<1>(NT, S, false, T, pk, small, nbal, m, din, dout, L, st);
    }
  }
  for (int k = 0; k < njobs; ++k) {
    const InsrJetJob& j = jobs[k];
    if (j.n == 0) continue;
    const int rc = insr_siren_jet_fwd(j.x, j.n, din, j.d_out > 0 ? j.d_out : dout, L, W, mode, j.params, j.y, j.dy,
                                      j.lap, j.act, stream);
    if (rc) return rc;
  }
  return 0;
}

// Host-side validation of a mixed launch's jobs, before anything touches the device.  Every
// field the kernel (jet_fwd_x6_mixed) indexes with is checked here: the job mode selects the
// body (an unknown mode runs nothing, but is refused first), d_out sizes the output rows, n the
// tiles / block ranges (first[] is built from n alone), and the advect job writes its foot and
// f(x) rows while other jobs of the same launch may read their x: those buffers must not alias
// any job's input.  (Round-2 record: an aperture violation in this kernel came from a job
// layout whose x could point into LDS -- the backed-out in-kernel draw)
static int mixed_jobs_ok(const InsrJetJob* jobs, const int* modes, const float* scalars, int njobs, int din, int dout,
                         int L, int W, int prec_mode, long* total_out) {
  if (!jobs || !modes || njobs < 1 || njobs > INSR_MAX_FWD_JOBS) return 0;
  if (prec_mode & INSR_MODE_MASK) return 0;  // the per-job jet modes come from `modes`
  long total = 0;
  for (int k = 0; k < njobs; ++k) {
    const InsrJetJob& j = jobs[k];
    const int md = modes[k];
    if (md != INSR_MODE_VALUE && md != INSR_MODE_GRAD && md != INSR_MODE_LAP && md != INSR_MIX_ADVECT) return 0;
    if (j.d_out < 0 || j.d_out > 3) return 0;
    const int dk = j.d_out > 0 ? j.d_out : dout;
    if (j.n < 0 || j.n > 0x7fffffffL || (j.n > 0 && (!j.x || !j.params || !j.y))) return 0;
    if (md == INSR_MIX_ADVECT) {  // two value jets + the foot: f maps R^d -> R^d
      if (dk != din || !scalars || !shape_ok(din, dk, L, W, INSR_MODE_VALUE | prec_mode)) return 0;
      if (j.n > 0) {
        if (!j.dy || !j.lap || j.dy == j.lap || j.dy == j.y || j.lap == j.y) return 0;
        for (int q = 0; q < njobs; ++q)  // the foot / f(x) rows must not alias an input of the launch
          if (jobs[q].n > 0 && (jobs[q].x == j.dy || jobs[q].x == j.lap)) return 0;
      }
    } else {
      if (!shape_ok(din, dk, L, W, md | prec_mode)) return 0;
      if (j.n > 0 && md != INSR_MODE_VALUE && !j.dy) return 0;
      if (j.n > 0 && md == INSR_MODE_LAP && !j.lap) return 0;
    }
    total += j.n;
  }
  if (total > 0x7fffffffL) return 0;
  *total_out = total;
  return 1;
}

int insr_siren_jet_fwd_mixed(const InsrJetJob* jobs, const int* modes, const float* scalars, int njobs, int din,
                             int dout, int L, int W, int prec_mode, void* stream) {
  long total = 0;
  if (!mixed_jobs_ok(jobs, modes, scalars, njobs, din, dout, L, W, prec_mode, &total)) return INSR_EINVAL;
  const JetCall c(din, W, INSR_MODE_VALUE | prec_mode);
  hipStream_t st = (hipStream_t)stream;
  if (c.NT == 8 && c.nqf > 0) {
    InsrJetJob pk[INSR_MAX_FWD_JOBS];
    int md[INSR_MAX_FWD_JOBS];
    int m = 0;
    for (int k = 0; k < njobs; ++k) {
      if (jobs[k].n == 0) continue;
      pk[m] = jobs[k];
      md[m] = modes[k];
      int rc = 0;
      const int dk = jobs[k].d_out > 0 ? jobs[k].d_out : dout;
      if (!(pk[m].params = with_planes(jobs[k].params, din, dk, L, W, prec_mode, st, k, &rc))) return rc;
      ++m;
    }
    if (m == 0) return 0;
    float sc[3 * INSR_MAX_FWD_JOBS] = {};
    for (int k = 0, q = 0; k < njobs; ++k)
      if (jobs[k].n > 0) {
        for (int r = 0; r < 3; ++r) sc[3 * q + r] = scalars ? scalars[3 * k + r] : 0.f;
        ++q;
      }
    switch (c.nqf) {
      case 4: return dispatch_fwd_mixed_q<4>(c.NT, din, pk, md, sc, m, dout, L, st);
      case 3: return dispatch_fwd_mixed_q<3>(c.NT, din, pk, md, sc, m, dout, L, st);
      case 2: return dispatch_fwd_mixed_q<2>(c.NT, din, pk, md, sc, m, dout, L, st);
      default: return dispatch_fwd_mixed_q<1>(c.NT, din, pk, md, sc, m, dout, L, st);
    }
  }
  for (int k = 0; k < njobs; ++k) {  // other widths / exact fp32: one launch per job
    const InsrJetJob& j = jobs[k];
    if (j.n == 0) continue;
    if (modes[k] == INSR_MIX_ADVECT) {  // f(x), the foot, f(foot)
      int rc = insr_siren_jet_fwd(j.x, j.n, din, din, L, W, INSR_MODE_VALUE | prec_mode, j.params, j.dy, nullptr,
                                  nullptr, nullptr, stream);
      if (!rc) rc = insr_axpy_clamp(j.x, j.dy, -scalars[3 * k], scalars[3 * k + 1], scalars[3 * k + 2], j.lap,
                                    j.n * din, stream);
      if (!rc) rc = insr_siren_jet_fwd(j.lap, j.n, din, din, L, W, INSR_MODE_VALUE | prec_mode, j.params, j.y,
                                       nullptr, nullptr, nullptr, stream);
      if (rc) return rc;
      continue;
    }
    const int rc = insr_siren_jet_fwd(j.x, j.n, din, j.d_out > 0 ? j.d_out : dout, L, W, modes[k] | prec_mode,
                                      j.params, j.y, j.dy, j.lap, j.act, stream);
    if (rc) return rc;
  }
  return 0;
}

static int bwd_fused_impl(const float* x, long n, int din, int dout, int L, int W, int mode, const float* params,
                          const float* act, const float* gy, const float* gdy, const float* glap, float* partial,
                          const SeedTab* seeds, void* stream) {
  if (!shape_ok(din, dout, L, W, mode) || n < 0 || n > 0x7fffffffL) return INSR_EINVAL;
  if (n == 0) return 0;
  if (!x || !params || !act || !partial) return INSR_EINVAL;
  const JetCall c(din, W, mode);
  const long P = insr_jet_partial_stride(din, dout, L, W);  // row stride of the partial rows
  // width 256: the fused split-bf16 backward does not exist -- exact fp32 serves this entry
  const int nq = c.NT > 8 ? 0 : c.nqb;
  const LaunchShape sh = launch_shape(1, nq, c.NT, c.S, c.lap, n, c.k);
  int rc = 0;
  if (nq > 0 && !(params = with_planes(params, din, dout, L, W, mode, (hipStream_t)stream, 0, &rc))) return rc;
  BwdJobsX6 J{};
  J.x[0] = x;
  J.act[0] = act;
  J.gy[0] = gy;
  J.gdy[0] = gdy;
  J.glap[0] = glap;
  J.n[0] = (int)n;
  J.nbal[0] = sh.nbal;
  J.first[0] = 0;
  J.first[1] = sh.nbal > 0 ? sh.nbal : (int)(((n + 15) / 16 + sh.T - 1) / sh.T);
  J.njobs = 1;
  if (seeds) {
    if (nq == 0) return INSR_EINVAL;  // the exact-fp32 kernel takes no seeds
    J.seeds = *seeds;
  }
  return bwd_q(fused_bwd_nq(nq, c.k), c.NT, c.S, c.lap, sh.T, &J, din, dout, L, params, partial, P, (hipStream_t)stream);
}

int insr_siren_jet_bwd(const float* x, long n, int din, int dout, int L, int W, int mode, const float* params,
                       const float* act, const float* gy, const float* gdy, const float* glap, float* partial,
                       void* stream) {
  return bwd_fused_impl(x, n, din, dout, L, W, mode, params, act, gy, gdy, glap, partial, nullptr, stream);
}

// Plan of a multi-job backward (insr_siren_jet_bwd_grad_multi): the jobs whose own size takes the
// fused tile-split path share one launch, T from the launch shape of their combined batch; a
// balanced shape (T = 3 / 5) gives each job its share of the balanced block count (never fewer
// blocks than T-tile blocks need); every other job runs alone on its own path.
namespace {
struct MultiPlan {
  int nq, T, nf, ns, nb;
  int fused[kBwdJobs], solo[kBwdJobs], blocks[kBwdJobs], nbal[kBwdJobs];
};
}  // namespace

static int plan_multi(const long* n, int njobs, int din, int dout, int L, int W, int mode, MultiPlan& p) {
  if (!n || njobs < 1 || njobs > kBwdJobs || !shape_ok(din, dout, L, W, mode)) return INSR_EINVAL;
  const JetCall c(din, W, mode);
  p = MultiPlan{};
  p.nq = c.NT > 8 ? 0 : c.nqb;
  long total = 0, tiles = 0;
  for (int k = 0; k < njobs; ++k) {
    if (n[k] < 0 || n[k] > 0x7fffffffL) return INSR_EINVAL;
    if (n[k] == 0) continue;
    if (p.nq > 0 && c.path(n[k], L) == 0) {
      p.fused[p.nf++] = k;
      total += n[k];
      tiles += (n[k] + 15) / 16;
    } else {
      p.solo[p.ns++] = k;
    }
  }
  if (total > 0x7fffffffL) return INSR_EINVAL;
  if (p.nf == 0) return 0;
  const LaunchShape sh = launch_shape(1, p.nq, c.NT, c.S, c.lap, total, c.k);
  p.T = sh.T;
  for (int q = 0; q < p.nf; ++q) {
    const long tk = (n[p.fused[q]] + 15) / 16, plain = (tk + sh.T - 1) / sh.T;
    long nbk = plain;
    if (sh.nbal > 0) {
      const long share = (tk * sh.nbal + tiles / 2) / tiles;
      nbk = share > plain ? share : plain;
    }
    p.blocks[q] = (int)nbk;
    p.nbal[q] = sh.nbal > 0 ? (int)nbk : 0;
    p.nb += (int)nbk;
  }
  return 0;
}

long insr_jet_bwd_multi_work_bytes(const long* n, int njobs, int din, int dout, int L, int W, int mode) {
  MultiPlan p;
  const int rc = plan_multi(n, njobs, din, dout, L, W, mode, p);
  if (rc) return rc;
  if (JetCall(din, W, mode).recompute(L)) {
    long tiles = 0;
    for (int k = 0; k < njobs; ++k) tiles += n[k] > 0 ? (n[k] + 15) / 16 : 0;
    return fb_work_floats(tiles, din, dout, L) * (long)sizeof(float);
  }
  long bytes = (long)p.nb * insr_jet_partial_stride(din, dout, L, W) * (long)sizeof(float);
  for (int q = 0; q < p.ns; ++q) {
    const long b = insr_jet_bwd_work_bytes(n[p.solo[q]], din, dout, L, W, mode);
    if (b < 0) return b;
    if (b > bytes) bytes = b;
  }
  return bytes;
}

static int wide_bwd_jobs(const JetCall& c, const FbJobs& J, long N, int din, int dout, int L, int W, int mode,
                         const float* params, float* work, float* grad, int accumulate, int phases, const AdamArgs& A,
                         hipStream_t st);
static int multi_fused_rows(const InsrBwdJob* jobs, const MultiPlan& p, int din, int dout, int L, int W, int mode,
                            const float* params, float* work, hipStream_t st);

int insr_siren_jet_bwd_grad_multi(const InsrBwdJob* jobs, int njobs, int din, int dout, int L, int W, int mode,
                                  const float* params, float* work, float* grad, int accumulate, void* stream) {
  if (!jobs || njobs < 1 || njobs > kBwdJobs) return INSR_EINVAL;
  long ns[kBwdJobs];
  const bool fb = shape_ok(din, dout, L, W, mode) && JetCall(din, W, mode).recompute(L);
  for (int k = 0; k < njobs; ++k) {
    ns[k] = jobs[k].n;
    if (jobs[k].n > 0 && (!jobs[k].x || (!jobs[k].act && !fb))) return INSR_EINVAL;
  }
  MultiPlan p;
  int rc = plan_multi(ns, njobs, din, dout, L, W, mode, p);
  if (rc) return rc;
  if (p.nf + p.ns == 0) return 0;
  if (!params || !work || !grad) return INSR_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  int acc = accumulate ? 1 : 0;
  {
    const JetCall c(din, W, mode);
    if (c.recompute(L)) {  // every job in ONE recompute launch (act is not read)
      FbJobs J{};
      int m = 0, t = 0;
      for (int k = 0; k < njobs; ++k) {
        if (jobs[k].n <= 0) continue;
        J.x[m] = jobs[k].x;
        J.gy[m] = jobs[k].gy;
        J.gdy[m] = jobs[k].gdy;
        J.glap[m] = jobs[k].glap;
        J.n[m] = (int)jobs[k].n;
        J.tstart[m] = t;
        t += (int)((jobs[k].n + 15) / 16);
        ++m;
      }
      J.tstart[m] = t;
      J.njobs = m;
      const float* prm = params;
      if (!(prm = with_planes(params, din, dout, L, W, mode, st, 0, &rc))) return rc;
      return dispatch_fb_bwd(c.S, c.lap, L, J, din, dout, prm, work, grad, acc, 0, 3, AdamArgs{}, st);
    }
  }
  if (p.nf > 0) {
    if ((rc = multi_fused_rows(jobs, p, din, dout, L, W, mode, params, work, st))) return rc;
    if ((rc = insr_reduce_partials_strided(work, p.nb, insr_siren_param_count(din, dout, L, W),
                                           insr_jet_partial_stride(din, dout, L, W), grad, acc, stream)))
      return rc;
    acc = 1;
  }
  for (int q = 0; q < p.ns; ++q) {  // stream order: the previous job's reduction has read `work`
    const InsrBwdJob& jb = jobs[p.solo[q]];
    if ((rc = insr_siren_jet_bwd_grad(jb.x, jb.n, din, dout, L, W, mode, params, jb.act, jb.gy, jb.gdy, jb.glap, work,
                                      grad, acc, stream)))
      return rc;
    acc = 1;
  }
  return 0;
}

int insr_siren_jet_bwd_multi_rows(const InsrBwdJob* jobs, int njobs, int din, int dout, int L, int W, int mode,
                                  const float* params, float* work, void* stream) {
  if (!jobs || njobs < 1 || njobs > kBwdJobs) return INSR_EINVAL;
  long ns[kBwdJobs];
  for (int k = 0; k < njobs; ++k) {
    ns[k] = jobs[k].n;
    if (jobs[k].n > 0 && (!jobs[k].x || !jobs[k].act)) return INSR_EINVAL;
  }
  MultiPlan p;
  int rc = plan_multi(ns, njobs, din, dout, L, W, mode, p);
  if (rc) return rc;
  if (p.ns > 0 || JetCall(din, W, mode).recompute(L)) return INSR_EINVAL;  // a job another path serves
  if (p.nf == 0) return 0;
  if (!params || !work) return INSR_EINVAL;
  if ((rc = multi_fused_rows(jobs, p, din, dout, L, W, mode, params, work, (hipStream_t)stream))) return rc;
  return p.nb;
}

int insr_siren_jet_bwd_multi_sweep(const InsrBwdJob* jobs, int njobs, int din, int dout, int L, int W, int mode,
                                   const float* params, float* work, void* stream) {
  if (!jobs || njobs < 1 || njobs > kBwdJobs || !shape_ok(din, dout, L, W, mode)) return INSR_EINVAL;
  const JetCall c(din, W, mode);
  long total = 0, tiles = 0;
  for (int k = 0; k < njobs; ++k) {
    if (jobs[k].n < 0 || jobs[k].n > 0x7fffffffL) return INSR_EINVAL;
    if (jobs[k].n > 0 && (!jobs[k].x || !jobs[k].act)) return INSR_EINVAL;
    total += jobs[k].n;
    tiles += (jobs[k].n + 15) / 16;
  }
  // the saved-stream resident sweep (jet_fb.hpp, f16x3) or -- round 6 -- the two-kernel backward (jet_x6w.hpp,
  // e.g. elasticity's interior batch + constraint bands, elasticity/model.py:137,161-174) must be the path of the
  // jobs' total; the two-kernel jobs are laid out over npass = 16 x their tiles, and phase 2 (the sums, with the
  // Adam launch: insr_siren_jet_bwd_grad_adam phases 2 at n = npass) finds them there
  const long npass = 16 * tiles;
  const bool fbp = !c.recompute(L) && c.resident(total, L) && c.resident_f16(total, L);
  const bool widep = !fbp && !c.recompute(L) && L > 0 && !c.resident(npass, L) && c.wide(npass);
  if (total > 0x7fffffffL || npass > 0x7fffffffL || !(fbp || widep)) return INSR_EINVAL;
  if (tiles == 0) return 0;
  if (!params || !work) return INSR_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  int rc = 0;
  const float* prm = params;
  if (!(prm = with_planes(params, din, dout, L, W, mode, st, 0, &rc))) return rc;
  FbJobs J{};
  int m = 0, t = 0;
  for (int k = 0; k < njobs; ++k) {
    if (jobs[k].n <= 0) continue;
    J.x[m] = jobs[k].x;
    J.act[m] = jobs[k].act;
    J.gy[m] = jobs[k].gy;
    J.gdy[m] = jobs[k].gdy;
    J.glap[m] = jobs[k].glap;
    J.n[m] = (int)jobs[k].n;
    J.tstart[m] = t;
    t += (int)((jobs[k].n + 15) / 16);
    ++m;
  }
  J.tstart[m] = t;
  J.njobs = m;
  if (widep) return wide_bwd_jobs(c, J, npass, din, dout, L, W, mode, params, work, nullptr, 0, 1, AdamArgs{}, st);
  return dispatch_fb_bwd(c.S, c.lap, L, J, din, dout, prm, work, nullptr, 0, 1, 1, AdamArgs{}, st);
}

// the multi plan's fused tile-split jobs in ONE jet_bwd_x6 launch: p.nb partial-gradient rows into work
static int multi_fused_rows(const InsrBwdJob* jobs, const MultiPlan& p, int din, int dout, int L, int W, int mode,
                            const float* params, float* work, hipStream_t st) {
  int rc = 0;
  {
    const JetCall c(din, W, mode);
    const float* prm = params;
    if (!(prm = with_planes(params, din, dout, L, W, mode, st, 0, &rc))) return rc;
    BwdJobsX6 J{};
    int b = 0;
    for (int q = 0; q < p.nf; ++q) {
      const InsrBwdJob& jb = jobs[p.fused[q]];
      J.x[q] = jb.x;
      J.act[q] = jb.act;
      J.gy[q] = jb.gy;
      J.gdy[q] = jb.gdy;
      J.glap[q] = jb.glap;
      J.n[q] = (int)jb.n;
      J.nbal[q] = p.nbal[q];
      J.first[q] = b;
      b += p.blocks[q];
    }
    J.first[p.nf] = b;
    J.njobs = p.nf;
    const long P = insr_jet_partial_stride(din, dout, L, W);
    return bwd_q(fused_bwd_nq(p.nq, c.k), c.NT, c.S, c.lap, p.T, &J, din, dout, L, prm, work, P, st);
  }
}

long insr_jet_bwd_work_bytes(long n, int din, int dout, int L, int W, int mode) {
  if (!shape_ok(din, dout, L, W, mode) || n < 0) return INSR_EINVAL;
  const JetCall c(din, W, mode);
  if (c.recompute(L) || c.resident_f16(n, L)) return fb_work_floats((n + 15) / 16, din, dout, L) * (long)sizeof(float);
  if (c.resident(n, L)) return resident_work_floats(n, din, dout, L) * (long)sizeof(float);
  if (c.wide(n)) return wide_work_floats(n, din, dout, L, W, c.S) * (long)sizeof(float);
  return insr_jet_partial_bytes(n, din, dout, L, W, mode);
}

int insr_jet_wide_launch_threads(long n, int din, int dout, int L, int W, int mode, long* threads3) {
  if (!shape_ok(din, dout, L, W, mode) || n <= 0 || !threads3 || L < 1) return INSR_EINVAL;
  const JetCall c(din, W, mode);
  if (c.recompute(L) || c.resident(n, L)) {  // the persistent launch + the dW / compact-row sums
    const long Ps = (long)W * din + W + (long)L * W + (long)dout * W + dout;
    const long wq = ((long)W * W / 4 + 63) / 64, rows_x = (Ps + 63) / 64;
    threads3[0] = (long)((c.recompute(L) || c.resident_f16(n, L)) ? fb_launch_blocks((n + 15) / 16) : resident_blocks(n)) * 512;
    threads3[1] = (wq > rows_x ? wq : rows_x) * (L + 1) * 512;
    threads3[2] = 0;
    return 0;
  }
  if (!c.wide(n)) return INSR_EINVAL;
  wide_launch_threads(n, din, dout, L, W, c.S, threads3);
  return 0;
}

int insr_jet_bwd_is_wide(long n, int din, int W, int mode) {
  const JetCall c(din, W, mode);
  if (!c.ok() || n < 0) return INSR_EINVAL;
  return c.wide(n) ? 1 : 0;
}

int insr_jet_bwd_path(long n, int din, int dout, int L, int W, int mode) {
  if (!shape_ok(din, dout, L, W, mode) || n < 0) return INSR_EINVAL;
  return JetCall(din, W, mode).path(n, L);
}

int insr_jet_bwd_kernel(long n, int din, int dout, int L, int W, int mode) {
  if (!shape_ok(din, dout, L, W, mode) || n < 0) return INSR_EINVAL;
  const JetCall c(din, W, mode);
  const int p = c.path(n, L);
  return (p == 3 || (p == 2 && c.resident_f16(n, L))) ? 1 : 0;
}

// The two-kernel (wide) backward of a job table laid out over N points (jet_x6w.hpp wide_bwd_t)
static int wide_bwd_jobs(const JetCall& c, const FbJobs& J, long N, int din, int dout, int L, int W, int mode,
                         const float* params, float* work, float* grad, int accumulate, int phases, const AdamArgs& A,
                         hipStream_t st) {
  int rc = 0;
  if (!(params = with_planes(params, din, dout, L, W, mode, st, 0, &rc))) return rc;
  switch (c.nqb) {
    case 3: return dispatch_wide_bwd_q<3>(c.NT, c.S, c.lap, J, (int)N, din, dout, L, params, work, grad, accumulate, c.k.f16, phases, A, st);
    case 2: return dispatch_wide_bwd_q<2>(c.NT, c.S, c.lap, J, (int)N, din, dout, L, params, work, grad, accumulate, c.k.f16, phases, A, st);
    default: return dispatch_wide_bwd_q<1>(c.NT, c.S, c.lap, J, (int)N, din, dout, L, params, work, grad, accumulate, c.k.f16, phases, A, st);
  }
}

// The two-kernel (wide) backward of one call: phases / Adam epilogue as wide_bwd_t
static int wide_bwd_call(const JetCall& c, const float* x, long n, int din, int dout, int L, int W, int mode,
                         const float* params, const float* act, const float* gy, const float* gdy, const float* glap,
                         float* work, float* grad, int accumulate, int phases, const AdamArgs& A, hipStream_t st) {
  FbJobs J{};
  J.x[0] = x;
  J.act[0] = act;
  J.gy[0] = gy;
  J.gdy[0] = gdy;
  J.glap[0] = glap;
  J.n[0] = (int)n;
  J.tstart[0] = 0;
  J.tstart[1] = (int)((n + 15) / 16);
  J.njobs = 1;
  return wide_bwd_jobs(c, J, n, din, dout, L, W, mode, params, work, grad, accumulate, phases, A, st);
}

// The single-job call of the jet_fb.hpp backward (the recompute kernel, or the resident sweep on the
// saved streams): phases / Adam epilogue as fb_bwd_t
static int fb_bwd_call(const JetCall& c, const float* x, long n, int din, int dout, int L, int W, int mode,
                       const float* params, const float* act, const float* gy, const float* gdy, const float* glap,
                       float* work, float* grad, int accumulate, int phases, const AdamArgs& A, hipStream_t st,
                       const SeedTab* seeds = nullptr) {
  int rc = 0;
  if (!(params = with_planes(params, din, dout, L, W, mode, st, 0, &rc))) return rc;
  FbJobs J{};
  if (seeds) J.seeds = *seeds;
  J.x[0] = x;
  J.act[0] = c.recompute(L) ? nullptr : act;
  J.gy[0] = gy;
  J.gdy[0] = gdy;
  J.glap[0] = glap;
  J.n[0] = (int)n;
  J.tstart[0] = 0;
  J.tstart[1] = (int)((n + 15) / 16);
  J.njobs = 1;
  return dispatch_fb_bwd(c.S, c.lap, L, J, din, dout, params, work, grad, accumulate, c.recompute(L) ? 0 : 1, phases,
                         A, st);
}

// InsrLossFin -> the device descriptor (NULL: none)
static int fin_of(const InsrLossFin* f, LossFin& F) {
  F = LossFin{};
  if (!f) return 0;
  if (!f->part || f->rows < 1 || f->nloss < 1 || f->nloss > INSR_SEED_MAX) return INSR_EINVAL;
  F.part = f->part;
  F.rows = f->rows;
  F.nloss = f->nloss;
  for (int k = 0; k < f->nloss; ++k) {
    if (!f->out[k]) return INSR_EINVAL;
    F.scale[k] = f->scale[k];
    F.out[k] = f->out[k];
  }
  return 0;
}

static int grad_adam_impl(const float* x, long n, int din, int dout, int L, int W, int mode, float* params,
                          const float* act, const float* gy, const float* gdy, const float* glap, float* work,
                          float* grad, int accumulate, int phases, float* exp_avg, float* exp_avg_sq, float* opt_state,
                          float beta1, float beta2, float eps, const float* loss, int patience, const LossFin& fin,
                          const SeedTab* seeds, void* stream) {
  if (!shape_ok(din, dout, L, W, mode) || n < 1 || n > 0x7fffffffL || phases < 1 || phases > 3) return INSR_EINVAL;
  const JetCall c(din, W, mode);
  const bool fb = c.recompute(L) || (c.resident(n, L) && c.resident_f16(n, L));  // jet_fb.hpp's backward
  const bool wide = !fb && !c.resident(n, L) && c.wide(n) && L > 0;               // the two-kernel backward
  if (!fb && !wide) return INSR_EINVAL;
  if (!params || !work || !grad) return INSR_EINVAL;
  if ((phases & 1) && (!x || (!act && !c.recompute(L)))) return INSR_EINVAL;  // the sweep's inputs
  AdamArgs A;
  if ((phases & 2) && exp_avg) {
    if (!exp_avg_sq || !opt_state) return INSR_EINVAL;
    A.p = params;
    A.m = exp_avg;
    A.v = exp_avg_sq;
    A.st = opt_state;
    A.loss = loss;
    A.patience = patience;
    A.b1 = beta1;
    A.b2 = beta2;
    A.eps = eps;
    if (mode & INSR_MODE_WSPLIT) {  // the buffer carries the weight planes: the update rewrites them
      A.shape[0] = din;
      A.shape[1] = dout;
      A.shape[2] = L;
      A.shape[3] = W;
    }
  }
  A.fin = fin;
  if ((fin.nloss && !(phases & 2)) || ((seeds || fin.nloss) && (wide || c.recompute(L)))) return INSR_EINVAL;
  if (wide)
    return wide_bwd_call(c, x, n, din, dout, L, W, mode, params, act, gy, gdy, glap, work, grad, accumulate, phases,
                         A, (hipStream_t)stream);
  return fb_bwd_call(c, x, n, din, dout, L, W, mode, params, act, gy, gdy, glap, work, grad, accumulate, phases, A,
                     (hipStream_t)stream, seeds);
}

int insr_siren_jet_bwd_grad_adam(const float* x, long n, int din, int dout, int L, int W, int mode, float* params,
                                 const float* act, const float* gy, const float* gdy, const float* glap, float* work,
                                 float* grad, int accumulate, int phases, float* exp_avg, float* exp_avg_sq,
                                 float* opt_state, float beta1, float beta2, float eps, const float* loss, int patience,
                                 void* stream) {
  return grad_adam_impl(x, n, din, dout, L, W, mode, params, act, gy, gdy, glap, work, grad, accumulate, phases,
                        exp_avg, exp_avg_sq, opt_state, beta1, beta2, eps, loss, patience, LossFin{}, nullptr, stream);
}

int insr_siren_jet_bwd_grad_adam_fin(const float* x, long n, int din, int dout, int L, int W, int mode, float* params,
                                     float* work, float* grad, int accumulate, float* exp_avg, float* exp_avg_sq,
                                     float* opt_state, float beta1, float beta2, float eps, const float* loss,
                                     int patience, const InsrLossFin* fin, void* stream) {
  LossFin F;
  if (fin_of(fin, F)) return INSR_EINVAL;
  return grad_adam_impl(x, n, din, dout, L, W, mode, params, nullptr, nullptr, nullptr, nullptr, work, grad,
                        accumulate, 2, exp_avg, exp_avg_sq, opt_state, beta1, beta2, eps, loss, patience, F, nullptr,
                        stream);
}

// InsrSeed[] -> the device table of a one-job launch (job 0); rejects a seeded stream whose adjoint
// pointer is set, overlapping terms of one stream, and malformed terms
static int seeds_of(const InsrSeed* seeds, int ns, float* lpart, const float* gy, const float* gdy, const float* glap,
                    SeedTab& T) {
  T = SeedTab{};
  if (!seeds || ns < 1 || ns > INSR_SEED_MAX || !lpart) return INSR_EINVAL;
  for (int k = 0; k < ns; ++k) {
    const InsrSeed& q = seeds[k];
    if (!q.a || q.n < 0 || q.a_off < 0 || q.loss < 0 || q.loss >= INSR_SEED_MAX) return INSR_EINVAL;
    if (q.stream < INSR_SEED_VALUE || q.stream > INSR_SEED_LAP) return INSR_EINVAL;
    if ((q.stream == INSR_SEED_VALUE && gy) || (q.stream == INSR_SEED_GRAD && gdy) || (q.stream == INSR_SEED_LAP && glap))
      return INSR_EINVAL;
    if (q.kind == INSR_LOSS_COMBO) {
      if ((q.d && !q.c) || q.sb < 1 || q.sc < 1 || q.sd < 1) return INSR_EINVAL;
    } else if (q.kind == INSR_LOSS_BANDS) {
      if (q.m < 2 || q.b || q.c || q.d || q.a_off % q.m) return INSR_EINVAL;
    } else {
      return INSR_EINVAL;
    }
    const long hi = q.a_off + (q.kind == INSR_LOSS_COMBO ? q.n : 2 * q.n * q.m);
    for (int j = 0; j < k; ++j) {
      const InsrSeed& o = seeds[j];
      const long ohi = o.a_off + (o.kind == INSR_LOSS_COMBO ? o.n : 2 * o.n * o.m);
      if (o.stream == q.stream && q.a_off < ohi && o.a_off < hi) return INSR_EINVAL;
    }
    SeedTerm& t = T.t[k];
    t.a = q.a + q.a_off;
    t.b = q.b;
    t.c = q.c;
    t.d = q.d;
    t.alpha = q.alpha;
    t.beta = q.beta;
    t.gamma = q.gamma;
    t.delta = q.delta;
    t.sb = q.sb;
    t.sc = q.sc;
    t.sd = q.sd;
    t.n = q.n;
    t.a_off = q.a_off;
    t.g2 = 2.f * q.scale;
    t.kind = q.kind;
    t.m = q.m;
    t.job = 0;
    t.stream = q.stream;
    t.loss = q.loss;
  }
  T.nt = ns;
  T.lpart = lpart;
  return 0;
}

int insr_jet_bwd_seed_rows(long n, int din, int dout, int L, int W, int mode) {
  if (!shape_ok(din, dout, L, W, mode) || n < 0 || n > 0x7fffffffL) return INSR_EINVAL;
  if (n == 0) return 0;
  const JetCall c(din, W, mode);
  const int p = c.path(n, L);
  // the fused tile-split kernel stages seeds for value jets (jet_x6.hpp jet_bwd_x6, S = 1)
  if (p == 0) return (c.S == 1 && (c.NT > 8 ? 0 : c.nqb) > 0) ? insr_jet_partial_blocks(n, din, W, mode) : 0;
  if (p == 2 && c.resident_f16(n, L)) {  // jet_fb.hpp on the saved streams: its tiles per block staged in LDS
    const long tiles = (n + 15) / 16, nb = fb_launch_blocks(tiles);
    return (tiles + nb - 1) / nb <= kFbSeedTiles ? (int)nb : 0;
  }
  return 0;
}

int insr_siren_jet_bwd_seeded(const float* x, long n, int din, int dout, int L, int W, int mode, const float* params,
                              const float* act, const float* gy, const float* gdy, const float* glap,
                              const InsrSeed* seeds, int n_seeds, float* loss_part, float* work, void* stream) {
  if (insr_jet_bwd_seed_rows(n, din, dout, L, W, mode) <= 0) return INSR_EINVAL;
  SeedTab T;
  if (seeds_of(seeds, n_seeds, loss_part, gy, gdy, glap, T)) return INSR_EINVAL;
  if (!x || !params || !act || !work) return INSR_EINVAL;
  const JetCall c(din, W, mode);
  if (c.path(n, L) == 2)  // the jet_fb sweep (phase 1); phase 2: insr_siren_jet_bwd_grad_adam_fin
    return grad_adam_impl(x, n, din, dout, L, W, mode, const_cast<float*>(params), act, gy, gdy, glap, work, work, 0, 1,
                          nullptr, nullptr, nullptr, 0.f, 0.f, 0.f, nullptr, 0, LossFin{}, &T, stream);
  return bwd_fused_impl(x, n, din, dout, L, W, mode, params, act, gy, gdy, glap, work, &T, stream);
}

int insr_siren_jet_bwd_grad(const float* x, long n, int din, int dout, int L, int W, int mode, const float* params,
                            const float* act, const float* gy, const float* gdy, const float* glap, float* work,
                            float* grad, int accumulate, void* stream) {
  if (!shape_ok(din, dout, L, W, mode) || n < 0 || n > 0x7fffffffL) return INSR_EINVAL;
  if (n == 0) return 0;
  const JetCall c(din, W, mode);
  if (!x || !params || (!act && !c.recompute(L)) || !work || !grad) return INSR_EINVAL;
  if (c.recompute(L) || (c.resident(n, L) && c.resident_f16(n, L)))  // jet_fb.hpp: one job
    return fb_bwd_call(c, x, n, din, dout, L, W, mode, params, act, gy, gdy, glap, work, grad, accumulate, 3,
                       AdamArgs{}, (hipStream_t)stream);
  if (c.resident(n, L)) {
    hipStream_t st = (hipStream_t)stream;
    int rc = 0;
    if (!(params = with_planes(params, din, dout, L, W, mode, st, 0, &rc))) return rc;
    return dispatch_resident_bwd(c.S, c.lap, L, x, (int)n, din, dout, params, act, gy, gdy, glap, work, grad,
                                 accumulate, st);
  }
  if (c.wide(n))
    return wide_bwd_call(c, x, n, din, dout, L, W, mode, params, act, gy, gdy, glap, work, grad, accumulate, 3,
                         AdamArgs{}, (hipStream_t)stream);
  int rc = insr_siren_jet_bwd(x, n, din, dout, L, W, mode, params, act, gy, gdy, glap, work, stream);
  if (rc) return rc;
  return insr_reduce_partials_strided(work, insr_jet_partial_blocks(n, din, W, mode),
                                      insr_siren_param_count(din, dout, L, W), insr_jet_partial_stride(din, dout, L, W),
                                      grad, accumulate, stream);
}

int insr_jet_partial_blocks(long n, int din, int W, int mode) {
  const JetCall c(din, W, mode);
  if (!c.ok() || n < 0) return INSR_EINVAL;
  if (n == 0) return 0;
  const int nq = c.NT > 8 ? 0 : c.nqb;
  const LaunchShape sh = launch_shape(1, nq, c.NT, c.S, c.lap, n, c.k);
  return sh.nbal > 0 ? sh.nbal : (int)(((n + 15) / 16 + sh.T - 1) / sh.T);
}

int insr_jet_split_tiles(long n, int din, int W, int mode, int backward) {
  const JetCall c(din, W, mode);
  if (!c.ok() || n < 0) return INSR_EINVAL;
  const int nq = backward ? (c.NT > 8 ? 0 : c.nqb) : c.nqf;
  return launch_shape(backward ? 1 : 0, nq, c.NT, c.S, c.lap, n, c.k).T;
}

static int reduce_partials_impl(const float* partial, int nb, long count, long stride, float* grad, int accumulate,
                                const LossFin& fin, void* stream) {
  if (!partial || !grad || nb < 0 || count < 0 || stride < count) return INSR_EINVAL;
  if (count == 0) return 0;
  if (stride % 4 == 0 && ((uintptr_t)partial & 15) == 0) {
    // fin.nloss > 0: one more block (no columns of its own) finishes the seeded loss values
    const long blocks = (count + 255) / 256, fb = fin.nloss ? 1 : 0;
    // many rows: two levels, so ~4 blocks per CU stream rows instead of ~1 (and no grid
    // that overshoots 256 CUs by a few blocks)
    // (measured: pays from ~1024 rows -- 58 -> 50 us; at 256 / 512 rows the extra launch
    // costs more than it saves)
    int slices = 1;
    while (nb >= 1024 && slices < 16 && nb / (2 * slices) >= 64 && blocks * slices < 1024) slices *= 2;
    if (slices > 1) {
      const int R = (nb + slices - 1) / slices;
      hipLaunchKernelGGL(reduce_slices4_kernel, dim3((unsigned)blocks, slices), dim3(64 * kRed4Waves), 0,
                         (hipStream_t)stream, const_cast<float*>(partial), nb, R, count, stride);
      hipLaunchKernelGGL(reduce_partials4_kernel, dim3((unsigned)(blocks + fb)), dim3(64 * kRed4Waves), 0,
                         (hipStream_t)stream, partial, (nb + R - 1) / R, count, stride * R, grad, accumulate, fin);
      return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(reduce_partials4_kernel, dim3((unsigned)(blocks + fb)), dim3(64 * kRed4Waves), 0,
                       (hipStream_t)stream, partial, nb, count, stride, grad, accumulate, fin);
    return (int)hipGetLastError();
  }
  if (stride != count || fin.nloss) return INSR_EINVAL;
  return insr_reduce_partials(partial, nb, count, grad, accumulate, stream);
}

int insr_reduce_partials_strided(const float* partial, int nb, long count, long stride, float* grad, int accumulate,
                                 void* stream) {
  return reduce_partials_impl(partial, nb, count, stride, grad, accumulate, LossFin{}, stream);
}

int insr_reduce_partials_fin(const float* partial, int nb, long count, long stride, float* grad, int accumulate,
                             const InsrLossFin* fin, void* stream) {
  LossFin F;
  if (fin_of(fin, F)) return INSR_EINVAL;
  return reduce_partials_impl(partial, nb, count, stride, grad, accumulate, F, stream);
}

int insr_reduce_partials(const float* partial, int nb, long count, float* grad, int accumulate, void* stream) {
  if (!partial || !grad || nb < 0 || count < 0) return INSR_EINVAL;
  if (count == 0) return 0;
  const long blocks = (count + 63) / 64;
  hipLaunchKernelGGL(reduce_partials_kernel, dim3((unsigned)blocks), dim3(64 * kRedWaves), 0,
                     (hipStream_t)stream, partial, nb, count, grad, accumulate);
  return (int)hipGetLastError();
}

int insr_adam_prepare(float* st, float b1, float b2, void* stream) {
  if (!st) return INSR_EINVAL;
  hipLaunchKernelGGL(adam_prepare_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, st, b1, b2);
  return (int)hipGetLastError();
}

int insr_plateau_step(float* st, const float* loss, int patience, int advance_step, void* stream) {
  if (!st || (!loss && !advance_step)) return INSR_EINVAL;
  hipLaunchKernelGGL(plateau_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, st, loss, patience, advance_step);
  return (int)hipGetLastError();
}

static int adam_partials_impl(const float* partial, int nb, long stride, float* grad, int accumulate, float* params,
                              float* exp_avg, float* exp_avg_sq, long count, const int* shape, float* st, float b1,
                              float b2, float eps, const float* loss, int patience, const LossFin& fin,
                              void* stream) {
  if (!partial || !grad || !params || !exp_avg || !exp_avg_sq || !st || nb < 1 || nb >= 1024 || count < 1 ||
      stride < count || stride % 4 || ((uintptr_t)partial & 15))
    return INSR_EINVAL;
  int4 shp = make_int4(0, 0, 0, 0);
  if (shape && shape[2] > 0) {  // a SIREN flat buffer with weight planes: its shape must match its size
    if (!shape_ok(shape[0], shape[1], shape[2], shape[3], 0) ||
        count != insr_siren_param_count(shape[0], shape[1], shape[2], shape[3]))
      return INSR_EINVAL;
    shp = make_int4(shape[0], shape[1], shape[2], shape[3]);
  }
  const long blocks = (count + 255) / 256 + (fin.nloss ? 1 : 0);  // + the loss-finishing block
  hipLaunchKernelGGL(reduce_adam_kernel, dim3((unsigned)blocks), dim3(64 * kRed4Waves), 0, (hipStream_t)stream,
                     partial, nb, count, stride, grad, accumulate, params, exp_avg, exp_avg_sq, shp, st, b1, b2, eps,
                     loss, patience, fin);
  return (int)hipGetLastError();
}

int insr_adam_step_partials(const float* partial, int nb, long stride, float* grad, int accumulate, float* params,
                            float* exp_avg, float* exp_avg_sq, long count, const int* shape, float* st, float b1,
                            float b2, float eps, const float* loss, int patience, void* stream) {
  return adam_partials_impl(partial, nb, stride, grad, accumulate, params, exp_avg, exp_avg_sq, count, shape, st, b1,
                            b2, eps, loss, patience, LossFin{}, stream);
}

int insr_adam_step_partials_fin(const float* partial, int nb, long stride, float* grad, int accumulate, float* params,
                                float* exp_avg, float* exp_avg_sq, long count, const int* shape, float* st, float b1,
                                float b2, float eps, const float* loss, int patience, const InsrLossFin* fin,
                                void* stream) {
  LossFin F;
  if (fin_of(fin, F)) return INSR_EINVAL;
  return adam_partials_impl(partial, nb, stride, grad, accumulate, params, exp_avg, exp_avg_sq, count, shape, st, b1,
                            b2, eps, loss, patience, F, stream);
}

int insr_adam_step_multi(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                         float* const* exp_avg_sq, const long* sizes, const float* st, float b1, float b2,
                         float eps, int step_offset, void* stream) {
  return insr_adam_step_nets(count, params, grads, exp_avg, exp_avg_sq, sizes, nullptr, st, b1, b2, eps, step_offset,
                             stream);
}

static int adam_launch(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                       float* const* exp_avg_sq, const long* sizes, const int* shapes, float* st, float b1, float b2,
                       float eps, int step_offset, const float* loss, int patience, void* stream);

int insr_adam_step_nets(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                        float* const* exp_avg_sq, const long* sizes, const int* shapes, const float* st, float b1,
                        float b2, float eps, int step_offset, void* stream) {
  return adam_launch(count, params, grads, exp_avg, exp_avg_sq, sizes, shapes, const_cast<float*>(st), b1, b2, eps,
                     step_offset, nullptr, 0, stream);
}

int insr_adam_plateau_step_nets(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                                float* const* exp_avg_sq, const long* sizes, const int* shapes, float* st, float b1,
                                float b2, float eps, const float* loss, int patience, void* stream) {
  if (!loss) return INSR_EINVAL;
  return adam_launch(count, params, grads, exp_avg, exp_avg_sq, sizes, shapes, st, b1, b2, eps, 1, loss, patience,
                     stream);
}

static int adam_launch(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                       float* const* exp_avg_sq, const long* sizes, const int* shapes, float* st, float b1, float b2,
                       float eps, int step_offset, const float* loss, int patience, void* stream) {
  if (count < 1 || count > INSR_ADAM_MAX_TENSORS || !st) return INSR_EINVAL;
  AdamList L;
  L.loss = loss;
  L.patience = patience;
  L.count = count;
  L.start[0] = 0;
  for (int k = 0; k < count; ++k) {
    for (int q = 0; q < 4; ++q) L.shape[k][q] = shapes ? shapes[4 * k + q] : 0;
    if (L.shape[k][2] > 0) {  // a SIREN flat buffer with weight planes: its shape must match its size
      const int* sh = L.shape[k];
      if (!shape_ok(sh[0], sh[1], sh[2], sh[3], 0) || sizes[k] != insr_siren_param_count(sh[0], sh[1], sh[2], sh[3]))
        return INSR_EINVAL;
    }
    if (!params[k] || !grads[k] || !exp_avg[k] || !exp_avg_sq[k] || sizes[k] < 0) return INSR_EINVAL;
    L.p[k] = params[k];
    L.g[k] = grads[k];
    L.m[k] = exp_avg[k];
    L.v[k] = exp_avg_sq[k];
    L.n[k] = sizes[k];
    L.start[k + 1] = L.start[k] + sizes[k];
  }
  const long total = L.start[count];
  if (total == 0) return loss ? insr_plateau_step(st, loss, patience, 1, stream) : 0;
  long blocks = (total + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, L, st, b1, b2,
                     eps, step_offset);
  return (int)hipGetLastError();
}

int insr_adam_step(float* p, const float* g, float* m, float* v, long n, const float* st, float b1, float b2,
                   float eps, void* stream) {
  // single buffer, explicit-prepare convention (t = st[STEP])
  long sz = n;
  return insr_adam_step_multi(1, &p, &g, &m, &v, &sz, st, b1, b2, eps, 0, stream);
}

}  // extern "C"
