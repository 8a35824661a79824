// jet_fb.hpp -- the RECOMPUTE backward of W = 128 SIRENs (jet_fb_x6): one persistent launch in
// which every CU walks its share of the batch's 16-point tiles and, per tile, runs the forward
// Taylor jet AND the reverse jet back to back, so nothing per point goes to HBM -- no saved
// pre-activation streams (the forward of the same call skips them) and no z̄ round trip.  The
// weight gradients of all hidden layers stay in registers across the tile loop (as jet_x6r.hpp);
// each block writes its dW once, reduce_dw_kernel sums them in a fixed order.
//
// Why (round-3 profiles, fluid2Dtlgn's pressure Laplacian jet at 16,708 points): the saved-stream
// dataflow moves ~700 MB per backward (137 MB of saved streams written by the forward and read
// twice, 103 MB of z̄ written and read) and runs at ~4 TB/s, waiting 49-67 % of its cycles.  Here
// the algorithmic traffic is the points, the adjoint seeds and one dW partial per CU (L W^2 floats);
// the price is the forward's matrix work once more (3 instead of 2 GEMM passes per stream and
// layer), on the matrix cores that the saved-stream kernels left idle.
//
// Per tile (wave w owns row tile w = 16 neurons of every hidden layer; lane (g, c) rows
// 16 w + 4 g .. + 3 at point c):
//   forward   layer 0 on the VALU (K = d_in), layers 1..L: z_j = W_j h_{j-1} on the fp16 matrix
//             cores (f16x3: two fp16 terms per operand, three products), h_{j-1} from LDS planes
//             (point-major, each stream class scaled per tile by the power of two that maps its
//             block maximum into [2^14, 2^15): the tangent streams too -- no |t| < 2183 limit);
//             the z-streams of every hidden layer are kept: the deepest ZR layers in registers,
//             the others in LDS (fp32), layer 0 is recomputed from x in the backward;
//   reverse   output layer on the VALU from the seeds (gy, gdy, glap of the loss), then per layer
//             j = L..1: sine reverse (lane-local), z̄_j and h_{j-1} into LDS planes (z̄ scaled per
//             tile: the block's 2^e; h's tangent / Laplacian streams by their own 2^eh, the
//             matching z̄ streams by 2^-eh, so every dW product carries exactly 2^e),
//               dW_j += z̄_j h_{j-1}^T        (registers; the accumulator's own power of two is
//                                             moved to the tile's 2^e first -- exact)
//               h̄_{j-1} = W_j^T z̄_j          (f16 W^T planes, one fragment prefetched)
//             and the first layer on the VALU.  Biases, the first and the output layer
//             accumulate in LDS (one owner lane per entry: a fixed order).
// Reference semantics: loss.backward() (base/baseModel.py:73-78) through the jets of
// base/diff_ops.py:33-82 -- the math of jet_x6.hpp / jet_x6w.hpp, another summation order.
#pragma once
#include <type_traits>

#include "jet_x6w.hpp"

namespace insr {

constexpr int kFbSmallMax = 1412;  // compact floats for W = 128, d_in, d_out <= 3, L <= 4 (16-B multiple)

// Diagnostic phase stamps (build with -DINSR_STAMPS: the diag library, tools/diag_fb.py): s_memtime at
// the phase boundaries of the first 8 tiles of block 0, [wave][tile][point]; never in the product build
#ifdef INSR_STAMPS
constexpr int kFbStampPts = 32;
static __device__ unsigned long long g_fb_stamps[8 * 8 * kFbStampPts];
#define FB_STAMP(k)                                                                                     \
  do {                                                                                                 \
    if (blockIdx.x == 0 && lane == 0 && tile - t0 < 8)                                                 \
      g_fb_stamps[((wave * 8 + (tile - t0)) * kFbStampPts) + (k)] = __builtin_amdgcn_s_memtime();     \
  } while (0)
#else
#define FB_STAMP(k) \
  do {              \
  } while (0)
#endif

// LDS image of the kernel (bytes): P = point-major planes [s][term][16 p][W + 8] (+ pad): the
// forward's B operand h_{j-1} and the reverse's z̄_j; H = point-major planes of h_{j-1} (the dW B
// operand, read by transpose reads as the A operand); ZS = fp32 z-streams of hidden layers 1..NZL
// [layer][s][wave][lane]; SW = the small weights;
// then the compact accumulators, the tile's seeds [S][3][16] and the block-maximum slots [2][4][8]
template <int S, int L, int ZR, bool SAVED = false, bool SEED = false>
struct FbGeo {
  using BG = X6BwdGeo<4, 8>;
  static constexpr int NZL = (!SAVED && (L - ZR) > 0) ? (L - ZR) : 0;
  static constexpr size_t P_BYTES = (size_t)S * BG::ZSET * 2;
  static constexpr size_t H_BYTES = (size_t)S * BG::ZSET * 2;  // point-major as P (dW B via transpose reads)
  static constexpr size_t ZS_BYTES = (size_t)NZL * S * 8 * 64 * 16;
  // the tile-invariant small weights, staged once per block: W_0 (W x 3), b_0, the hidden biases
  // (L x W), W_out (3 x W) -- read per tile from LDS instead of global memory
  static constexpr int SW_FLOATS = 128 * 3 + 128 + L * 128 + 3 * 128;
  static constexpr size_t SW_OFF = P_BYTES + H_BYTES + ZS_BYTES;
  static constexpr size_t SACC_OFF = SW_OFF + (size_t)SW_FLOATS * 4;
  static constexpr size_t SEED_OFF = SACC_OFF + (size_t)kFbSmallMax * 4;
  static constexpr size_t MX_OFF = SEED_OFF + (size_t)S * 3 * 16 * 4;
  // in-kernel seeds (saved-stream variant): the adjoints of the block's tiles [tile][S][3][16] (at most
  // kFbSeedTiles tiles per block), then the waves' square sums [8][INSR_SEED_MAX]
  static constexpr size_t SSEED_OFF = MX_OFF + 2 * 5 * 8 * 4;
  static constexpr size_t BYTES = SSEED_OFF + (SEED ? ((size_t)kFbSeedTiles * S * 48 + 8 * INSR_SEED_MAX) * 4 : 0);
};

// sin / cos of w z (4 values).  A wave holding any |w z| > 8192 takes the libm path, out of line:
// inlined, its Payne-Hanek reduction would need its registers at every call site, next to the
// 128 dW accumulators (the call saves what it uses, on the rare path only)
struct FbSinCos {
  floatx4 s, c;
};
__device__ __noinline__ FbSinCos fb_sincos_libm(floatx4 z) {
  FbSinCos o;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float a, b;
    sincosf(OMEGA * z[r], &a, &b);
    o.s[r] = a;
    o.c[r] = b;
  }
  return o;
}
__device__ __forceinline__ void fb_sincos(const floatx4& z, floatx4& s, floatx4& c) {
  float amax = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) amax = fmaxf(amax, fabsf(OMEGA * z[r]));
  if (wave_any_big(amax)) {
    const FbSinCos o = fb_sincos_libm(z);
    s = o.s;
    c = o.c;
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float a, b;
    sincos_fast(OMEGA * z[r], a, b);
    s[r] = a;
    c[r] = b;
  }
}

// h-stream s of a sine layer from its z-streams (z[1..S-1]) and sin / cos
template <int S, bool LAP>
__device__ __forceinline__ floatx4 fb_h(int s, const floatx4 (&z)[S], const floatx4& sn, const floatx4& cs) {
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  if (s == 0) return sn;
  floatx4 out;
  if (LAP && s == S - 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float t2 = 0.f;
#pragma unroll
      for (int i = 0; i < NTAN; ++i) t2 = fmaf(z[1 + i][r], z[1 + i][r], t2);
      out[r] = OMEGA * cs[r] * z[S - 1][r] - OMEGA2 * sn[r] * t2;
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) out[r] = OMEGA * cs[r] * z[s][r];
  }
  return out;
}

// this lane's bounds of a sine layer's h-streams: tangents w |t|, Laplacian w |q| + w^2 sum t^2
template <int S, bool LAP>
__device__ __forceinline__ void fb_h_bounds(const floatx4 (&z)[S], float& mt, float& ml) {
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  mt = 0.f;
  ml = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float t2 = 0.f;
#pragma unroll
    for (int i = 0; i < NTAN; ++i) {
      t2 = fmaf(z[1 + i][r], z[1 + i][r], t2);
      mt = fmaxf(mt, fabsf(z[1 + i][r]));
    }
    if constexpr (LAP) ml = fmaxf(ml, fmaf(OMEGA, fabsf(z[S - 1][r]), OMEGA2 * t2));
  }
  mt *= OMEGA;
}

// SEED (saved streams only): the in-kernel adjoint seeds of FbJobs::seeds, a separate instantiation so the
// pointer-seeded kernel is unchanged
template <int S, bool LAP, int L, int ZR, bool SAVED, bool SEED = false>
__global__ __launch_bounds__(512, 1) void jet_fb_x6(const FbJobs J, int din, int dout, const float* __restrict__ prm,
                                                    float* __restrict__ dpart, float* __restrict__ small, long Ps,
                                                    int nb, int tiles) {
  constexpr int NT = 8, W = 128, KC = 4;
  using BG = X6BwdGeo<4, NT>;
  using GG = FbGeo<S, L, ZR, SAVED, SEED>;
  static_assert(!SEED || SAVED, "seeds: the saved-stream variant");
  constexpr int LDB = BG::ZROW, ZPLANE = BG::ZPLANE, ZSET = BG::ZSET;
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  constexpr int NZL = GG::NZL;
  constexpr int NCH = (S + 1) / 2;  // 32-deep K chunks of one tile's dW (S sets of 16 points)
  static_assert(ZR >= 1 && ZR <= L, "z of layer L in registers");
  extern __shared__ __attribute__((aligned(16))) float lds_f[];
  unsigned char* lb = reinterpret_cast<unsigned char*>(lds_f);
  float* sacc0 = reinterpret_cast<float*>(lb + GG::SACC_OFF);
  const int t0 = (int)((long)blockIdx.x * tiles / nb), t1 = (int)((long)(blockIdx.x + 1) * tiles / nb);
  const long sb = (long)W * din + W;  // compact offset of b_1 (small_count layout, jet_x6w.hpp)
  const long so = sb + (long)L * W;   // compact offset of W_out
  for (int i = threadIdx.x; i < Ps; i += 512) sacc0[i] = 0.f;
  {  // SW: [W_0 rows (3 per row, d_in used) | b_0 | b_1 .. b_L | W_out rows (W per output)]
    float* sw = reinterpret_cast<float*>(lb + GG::SW_OFF);
    for (int i = threadIdx.x; i < W * 3; i += 512) sw[i] = (i % 3) < din ? prm[(i / 3) * din + i % 3] : 0.f;
    for (int i = threadIdx.x; i < W; i += 512) sw[3 * W + i] = prm[(long)W * din + i];
    for (int i = threadIdx.x; i < L * W; i += 512) sw[4 * W + i] = prm[hidden_off(din, W, 1 + i / W) + (long)W * W + i % W];
    for (int i = threadIdx.x; i < dout * W; i += 512) sw[(4 + L) * W + i] = prm[out_off(din, W, L) + i];
  }

  floatx4 dacc[L][NT];
#pragma unroll
  for (int j = 0; j < L; ++j)
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) dacc[j][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
  int E[L];  // power of two the accumulator dacc[j] carries (kNoE: nothing accumulated yet)
  constexpr int kNoE = -100000;
#pragma unroll
  for (int j = 0; j < L; ++j) E[j] = kNoE;
  int slot = 0;  // block-maximum slot of the next exchange (two alternate: each exchange has a barrier)

  // In-kernel seeds (saved streams, J.seeds): the adjoints of all the block's tiles, formed before the
  // tile loop -- from their pointers or the loss terms (jet_common.hpp seed_adjoint, each element by one
  // thread, which counts the term's square) -- into LDS; the block's square sums into J.seeds.lpart
  if constexpr (SEED) {
    float* ss = reinterpret_cast<float*>(lb + GG::SSEED_OFF);
    float* swq = ss + kFbSeedTiles * S * 48;
    float sq[INSR_SEED_MAX] = {0.f, 0.f, 0.f, 0.f};
    if (J.njobs == 1) {
      // one job (the merged [interior; bands] batch): every element of the block's tiles in flat order,
      // up to 3 per thread per round with all their operand loads issued before any adjoint is formed
      const int total = (t1 - t0) * S * 48;
      for (int b0 = threadIdx.x; b0 < total; b0 += 3 * 512) {
        SeedOps ops[3];
        float pv[3];
        bool live[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int idx = b0 + u * 512, i = idx % (S * 48), tile = t0 + idx / (S * 48);
          const int s = i / 48, o = (i / 16) % 3, pp = tile * 16 + (i & 15);
          const int sk = s == 0 ? INSR_SEED_VALUE : ((LAP && s == S - 1) ? INSR_SEED_LAP : INSR_SEED_GRAD);
          const float* g0 = sk == INSR_SEED_VALUE ? J.gy[0] : (sk == INSR_SEED_LAP ? J.glap[0] : J.gdy[0]);
          const long at = sk != INSR_SEED_GRAD ? (long)pp * dout + o : ((long)pp * dout + o) * din + (s - 1);
          live[u] = idx < total && o < dout && pp < J.n[0];
          ops[u] = SeedOps{0.f, 0.f, 0.f, 0.f, -1};
          pv[u] = 0.f;
          if (live[u]) {
            if (g0)
              pv[u] = g0[at];
            else
              ops[u] = seed_gather(J.seeds, 0, sk, at);
          }
        }
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int idx = b0 + u * 512;
          if (idx >= total) continue;
          const int s = (idx % (S * 48)) / 48;
          const int sk = s == 0 ? INSR_SEED_VALUE : ((LAP && s == S - 1) ? INSR_SEED_LAP : INSR_SEED_GRAD);
          const float* g0 = sk == INSR_SEED_VALUE ? J.gy[0] : (sk == INSR_SEED_LAP ? J.glap[0] : J.gdy[0]);
          ss[idx] = (live[u] && !g0) ? seed_finish(J.seeds, ops[u], sq) : pv[u];
        }
      }
    } else {
      for (int tile = t0; tile < t1; ++tile) {  // tile-uniform: the job index stays scalar
        int k = 0;
#pragma unroll
        for (int q = 1; q < kBwdJobs; ++q) k += (q < J.njobs && tile >= J.tstart[q]) ? 1 : 0;
        const int i = threadIdx.x;
        if (i < S * 48) {
          const int s = i / 48, o = (i / 16) % 3, pp = (tile - J.tstart[k]) * 16 + (i & 15);
          float v = 0.f;
          if (o < dout && pp < J.n[k]) {
            const int sk = s == 0 ? INSR_SEED_VALUE : ((LAP && s == S - 1) ? INSR_SEED_LAP : INSR_SEED_GRAD);
            const float* g0 = sk == INSR_SEED_VALUE ? J.gy[k] : (sk == INSR_SEED_LAP ? J.glap[k] : J.gdy[k]);
            const long at = sk != INSR_SEED_GRAD ? (long)pp * dout + o : ((long)pp * dout + o) * din + (s - 1);
            v = g0 ? g0[at] : seed_adjoint(J.seeds, k, sk, at, true, sq);
          }
          ss[(tile - t0) * S * 48 + i] = v;
        }
      }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < INSR_SEED_MAX; ++q) {
      float v = sq[q];
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0) swq[wave * INSR_SEED_MAX + q] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      floatx4 r = floatx4{0.f, 0.f, 0.f, 0.f};
      for (int w = 0; w < 8; ++w)
#pragma unroll
        for (int q = 0; q < INSR_SEED_MAX; ++q) r[q] += swq[w * INSR_SEED_MAX + q];
      *reinterpret_cast<floatx4*>(J.seeds.lpart + (long)blockIdx.x * INSR_SEED_MAX) = r;
    }
  }

  __syncthreads();  // sacc zeroed (and the staged seeds written)

  for (int tile = t0; tile < t1; ++tile) {
    // the LDS images through an opaque per-tile offset: otherwise the compiler hoists every
    // tile-invariant LDS address of the unrolled body out of the loop, one VGPR each (spills)
    // (the same for the parameter pointer and the thread index: every address derived from them is
    // rematerialised inside the body instead of pinned in a register across the loop)
    int zo = 0, po = 0, tid = threadIdx.x;
    asm volatile("" : "+s"(zo), "+s"(po));
    asm volatile("" : "+v"(tid));
    const float* prmt = prm + po;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, g = lane >> 4, c = lane & 15;
    const int rt = wave;             // this wave's row tile of every hidden layer
    const int ra = wave >> 1, cb = wave & 1;  // its dW tiles: rows 2 ra, 2 ra + 1 x columns 4 cb .. 4 cb + 3
    const int n0 = 16 * rt + 4 * g;  // this lane's first neuron
    const u32x4* wsp = wsp_base(prmt, din, dout, L, W);
    unsigned char* lbt = lb + zo;
    unsigned short* P = reinterpret_cast<unsigned short*>(lbt);
    unsigned short* H = reinterpret_cast<unsigned short*>(lbt + GG::P_BYTES);
    floatx4* ZS = reinterpret_cast<floatx4*>(lbt + GG::P_BYTES + GG::H_BYTES);
    const float* sw = reinterpret_cast<const float*>(lbt + GG::SW_OFF);
    const float* W0s = sw;                    // W_0 row n at 3 n
    const float* b0s = sw + 3 * W;
    const float* bhs = sw + 4 * W;            // b_j at (j - 1) W
    const float* Wos = sw + (4 + L) * W;      // W_out row o at o W
    float* sacc = reinterpret_cast<float*>(lbt + GG::SACC_OFF);
    float* seed = reinterpret_cast<float*>(lbt + GG::SEED_OFF);
    float* mx = reinterpret_cast<float*>(lbt + GG::MX_OFF);
    // block maxima of NC (<= 5) classes of non-negative values: each wave's values in, the block's out
    // (wave-uniform); one barrier.  Slot [class][wave], two slots alternate (each exchange has a barrier)
    auto exchange = [&](float (&m)[5], auto ncls) __attribute__((always_inline)) {
      constexpr int NC = decltype(ncls)::value;
#pragma unroll
      for (int k = 0; k < NC; ++k) m[k] = wave_max_nn(m[k]);
      if (lane < NC) {
        float v = m[0];
#pragma unroll
        for (int k = 1; k < NC; ++k) v = lane == k ? m[k] : v;
        mx[(slot * 5 + lane) * 8 + wave] = v;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < NC; ++k) {
        const floatx4 a = *reinterpret_cast<const floatx4*>(mx + (slot * 5 + k) * 8);
        const floatx4 b = *reinterpret_cast<const floatx4*>(mx + (slot * 5 + k) * 8 + 4);
        const float v = fmaxf(fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3])), fmaxf(fmaxf(b[0], b[1]), fmaxf(b[2], b[3])));
        m[k] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
      }
      slot ^= 1;
    };

    int k = 0;
#pragma unroll
    for (int q = 1; q < kBwdJobs; ++q) k += (q < J.njobs && tile >= J.tstart[q]) ? 1 : 0;
    const int lt = tile - J.tstart[k];
    const int N = J.n[k];
    const int p = lt * 16 + c;
    const bool valid = p < N;
    const float* __restrict__ x = J.x[k];
    float xk[3];
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) xk[kk] = (valid && kk < din) ? x[(long)p * din + kk] : 0.f;
    FB_STAMP(0);
    // the tile's adjoint seeds.  Recompute: thread i -> (stream s, output o, point), issued now, in
    // flight under the forward, staged into LDS before its last barrier.  Saved streams (no forward):
    // every lane loads its own point's seeds
    float sdv = 0.f;
    float gsd[(SAVED && !SEED) ? S : 1][3];
    if constexpr (SAVED && !SEED) {
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int o = 0; o < 3; ++o) {
          float v = 0.f;
          if (valid && o < dout) {
            const float* g0 = s == 0 ? J.gy[k] : ((LAP && s == S - 1) ? J.glap[k] : J.gdy[k]);
            const long at = (s == 0 || (LAP && s == S - 1)) ? (long)p * dout + o : ((long)p * dout + o) * din + (s - 1);
            if (g0) v = g0[at];
          }
          gsd[s][o] = v;
        }
    }
    // z-streams of hidden layer `layer` (1..L) of this tile from the forward's saved streams
    // (act layout: [layer][tile][stream][row tile][lane][4], jet_common.hpp act_base)
    const float* actk = SAVED ? J.act[k] : nullptr;
    const int ntk = ((N + 63) / 64) * 4;
    auto zload = [&](int layer, floatx4 (&z)[S]) __attribute__((always_inline)) {
      const float* base = act_base(actk, layer, ntk, lt, S, NT);
#pragma unroll
      for (int s = 0; s < S; ++s) z[s] = *reinterpret_cast<const floatx4*>(base + ((s * NT + rt) * 64 + lane) * 4);
    };
    if constexpr (!SAVED) {
      const int i = tid, s = i / 48, o = (i / 16) % 3, pp = lt * 16 + (i & 15);
      if (s < S && o < dout && pp < N) {
        const float* gy = J.gy[k];
        const float* gdy = J.gdy[k];
        const float* glap = J.glap[k];
        if (s == 0)
          sdv = gy ? gy[(long)pp * dout + o] : 0.f;
        else if (LAP && s == S - 1)
          sdv = glap ? glap[(long)pp * dout + o] : 0.f;
        else
          sdv = gdy ? gdy[((long)pp * dout + o) * din + (s - 1)] : 0.f;
      }
    }

    floatx4 zr[SAVED ? 1 : ZR][S];  // z-streams of hidden layers NZL + 1 .. L (registers)
    int eh[L][2];  // per layer j < L: the powers of two of h_j's tangent / Laplacian planes (block-uniform)
    if constexpr (!SAVED) {
    // ---------------- forward ----------------
    floatx4 a[S];       // z-streams of the current layer
    // layer 0 (K = d_in: exact fp32 VALU); tangents = W_0 columns, Laplacian stream 0
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + r;
      float z = b0s[n];
#pragma unroll
      for (int kk = 0; kk < 3; ++kk)
        if (kk < din) z = fmaf(W0s[3 * n + kk], xk[kk], z);
      a[0][r] = z;
#pragma unroll
      for (int i = 0; i < NTAN; ++i) a[1 + i][r] = W0s[3 * n + i];
      if constexpr (LAP) a[S - 1][r] = 0.f;
    }
    // unscale of the next layer's products per stream class (value, tangents, Laplacian)
    float usv = 1.f / kF16WScale, ust = 1.f / kF16WScale, usl = 1.f / kF16WScale;
    // h_j of the current layer -> P planes (block scales per class); two barriers
    auto put_h = [&](auto jc, bool stage_seeds) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (S > 1) fb_h_bounds<S, LAP>(a, m[0], m[1]);
      if (stage_seeds && tid < S * 48) seed[tid] = sdv;
      // + every wave's reads of P (this layer's B operand) done
      exchange(m, std::integral_constant<int, (S > 1 ? (LAP ? 2 : 1) : 0)>{});
      const int et = f16_exp_for(m[0]), el = f16_exp_for(m[1]);
      eh[j][0] = et;  // h_j's tangent / Laplacian powers of two: the reverse's dW B operand reuses them
      eh[j][1] = el;
      const float sct = ldexpf(1.f, et), scl = ldexpf(1.f, el);
      ust = ldexpf(1.f, -et) / kF16WScale;
      usl = ldexpf(1.f, -el) / kF16WScale;
      floatx4 sn, cs;
      fb_sincos(a[0], sn, cs);
      const int col = c * LDB + n0;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        floatx4 h = fb_h<S, LAP>(s, a, sn, cs);
        if (s > 0) h *= (LAP && s == S - 1) ? scl : sct;
        lds_put4<4, ZPLANE>(P + s * ZSET + col, h[0], h[1], h[2], h[3]);
      }
      __syncthreads();
    };
    // each forward layer's first weight fragment is issued before the previous layer's plane phase
    // (two barriers of latency to cover its L2 fetch)
    FragQ<4> wpre = wsp_frag<4, NT>(wsp, L, 0, 1, rt, 0, lane);
    put_h(std::integral_constant<int, 0>{}, L == 1);
    FB_STAMP(1);
    auto fwd_layer = [&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const u32x4* wsl = wsp;  // (tile-invariant loads: wsp derives from the per-tile opaque offset)
      floatx4 acc[S];
      acc[0] = *reinterpret_cast<const floatx4*>(bhs + (j - 1) * W + n0) * kF16WScale;
#pragma unroll
      for (int s = 1; s < S; ++s) acc[s] = floatx4{0.f, 0.f, 0.f, 0.f};
      FragQ<4> wf = wpre;
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const FragQ<4> wc = wf;
        if (kc + 1 < KC) wf = wsp_frag<4, NT>(wsl, L, 0, j, rt, kc + 1, lane);
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const FragQ<4> bf = lds_frag<4, ZPLANE>(P + s * ZSET + c * LDB + 32 * kc + 8 * g);
          acc[s] = mfma_q<4>(wc, bf, acc[s]);
          X6_SCHED_FENCE();
        }
      }
#pragma unroll
      for (int s = 0; s < S; ++s) a[s] = acc[s] * (s == 0 ? usv : ((LAP && s == S - 1) ? usl : ust));
      FB_STAMP(2 * j);
      if constexpr (j <= NZL) {
#pragma unroll
        for (int s = 0; s < S; ++s) ZS[(((j - 1) * S + s) * 8 + wave) * 64 + lane] = a[s];
      } else {
#pragma unroll
        for (int s = 0; s < S; ++s) zr[j - NZL - 1][s] = a[s];
      }
      if constexpr (j < L) {
        wpre = wsp_frag<4, NT>(wsl, L, 0, j + 1, rt, 0, lane);
        put_h(jc, j == L - 1);
      }
      FB_STAMP(2 * j + 1);
    };
    if constexpr (L >= 1) fwd_layer(std::integral_constant<int, 1>{});
    if constexpr (L >= 2) fwd_layer(std::integral_constant<int, 2>{});
    if constexpr (L >= 3) fwd_layer(std::integral_constant<int, 3>{});
    if constexpr (L >= 4) fwd_layer(std::integral_constant<int, 4>{});
    }  // forward (recompute only)

    // ---------------- reverse ----------------
    // output layer (exact fp32 VALU): hb = W_out^T g, dW_out / db_out into the compact row
    floatx4 zc[S];  // z-streams of the current layer
    if constexpr (SAVED) {
      zload(L, zc);
    } else {
#pragma unroll
      for (int s = 0; s < S; ++s) zc[s] = zr[ZR - 1][s];
    }
    floatx4 sn, cs;
    fb_sincos(zc[0], sn, cs);
    floatx4 hb[S];
#pragma unroll
    for (int s = 0; s < S; ++s) hb[s] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int o = 0; o < dout; ++o) {
      float ga[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if constexpr (!SAVED)
          ga[s] = seed[(s * 3 + o) * 16 + c];
        else if constexpr (SEED)  // the block's staged seeds of this tile
          ga[s] = reinterpret_cast<const float*>(lbt + GG::SSEED_OFF)[(((tile - t0) * S + s) * 3 + o) * 16 + c];
        else
          ga[s] = o == 0 ? gsd[s][0] : (o == 1 ? gsd[s][1] : gsd[s][2]);
      }
      const floatx4 w4 = *reinterpret_cast<const floatx4*>(Wos + (o * W + n0));
      floatx4 acc4 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const floatx4 hs = fb_h<S, LAP>(s, zc, sn, cs);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc4[r] = fmaf(ga[s], hs[r], acc4[r]);
          hb[s][r] = fmaf(w4[r], ga[s], hb[s][r]);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = sum16(acc4[r]);
        if (c == 0) sacc[so + (long)o * W + n0 + r] += v;
      }
      if (wave == 0) {
        const float v = sum16(g == 0 ? ga[0] : 0.f);
        if (lane == 0) sacc[so + (long)dout * W + o] += v;
      }
    }

    FB_STAMP(10);
    auto bwd_layer = [&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      constexpr int sp = 11 + 5 * (L - j);
      const u32x4* wsl = wsp;
      // z-streams of layer j - 1 (layer 0: recomputed from x) and their sin / cos; the saved-stream
      // variant issues their loads here, under the sine reverse and the sums
      floatx4 zp[S];
      if constexpr (SAVED && j > 1) zload(j - 1, zp);
      sine_rev<S, LAP>(hb, zc, sn, cs);  // hb = z̄_j
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = sum16(hb[0][r]);
        if (c == 0) sacc[sb + (long)(j - 1) * W + n0 + r] += v;
      }
      if constexpr (j == 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + r;
          float z = b0s[n];
    #pragma unroll
      for (int kk = 0; kk < 3; ++kk)
        if (kk < din) z = fmaf(W0s[3 * n + kk], xk[kk], z);
          zp[0][r] = z;
#pragma unroll
          for (int i = 0; i < NTAN; ++i) zp[1 + i][r] = W0s[3 * n + i];
          if constexpr (LAP) zp[S - 1][r] = 0.f;
        }
      } else if constexpr (SAVED) {
        // loaded above
      } else if constexpr (j - 1 <= NZL) {
#pragma unroll
        for (int s = 0; s < S; ++s) zp[s] = ZS[(((j - 2) * S + s) * 8 + wave) * 64 + lane];
      } else {
#pragma unroll
        for (int s = 0; s < S; ++s) zp[s] = zr[j - 1 - NZL - 1][s];
      }
      // classes: |z̄| value, tangents, Laplacian; h_{j-1}'s bounds (tangents, Laplacian): the forward's
      // scales eh[j - 1], or (saved streams) this exchange's classes 3, 4
      float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int cl = s == 0 ? 0 : ((LAP && s == S - 1) ? 2 : 1);
          m[cl] = fmaxf(m[cl], fabsf(hb[s][r]));
        }
      if constexpr (SAVED && S > 1) fb_h_bounds<S, LAP>(zp, m[3], m[4]);
      FB_STAMP(sp);
      // + every wave's reads of P / H (the previous layer's / the forward's) done
      exchange(m, std::integral_constant<int, (S == 1 ? 1 : (SAVED ? 5 : (LAP ? 3 : 2)))>{});
      FB_STAMP(sp + 1);
      int eht = 0, ehl = 0;
      if constexpr (SAVED) {
        if constexpr (S > 1) eht = f16_exp_for(m[3]);
        if constexpr (LAP) ehl = f16_exp_for(m[4]);
      } else {
        if constexpr (S > 1) eht = eh[j - 1][0];
        if constexpr (LAP) ehl = eh[j - 1][1];
      }
      const float bht = ldexpf(1.f, eht), bhl = ldexpf(1.f, ehl);   // h's tangent / Laplacian scales
      const float zht = ldexpf(1.f, -eht), zhl = ldexpf(1.f, -ehl);  // ... and the matching z̄ factors
      int e = f16_exp_for(fmaxf(m[0], fmaxf(m[1] * zht, m[2] * zhl)));
      if (E[j - 1] != kNoE) {  // move the accumulator to the tile's power of two (uniform branch)
        e = min(e, E[j - 1] + 60);
        if (e != E[j - 1]) {
          const float f = ldexpf(1.f, e - E[j - 1]);
#pragma unroll
          for (int ct = 0; ct < NT; ++ct) dacc[j - 1][ct] *= f;
        }
      }
      E[j - 1] = e;
      const float zsc = ldexpf(1.f, e);
      const int col = c * LDB + n0;
      {
        floatx4 snp, csp;
        fb_sincos(zp[0], snp, csp);
#pragma unroll
        for (int s = 0; s < S; ++s) {
        const float f2 = s == 0 ? 1.f : ((LAP && s == S - 1) ? zhl : zht);
        const floatx4 v = (hb[s] * zsc) * f2;  // each factor within fp32's range
        lds_put4<4, ZPLANE>(P + s * ZSET + col, v[0], v[1], v[2], v[3]);
          floatx4 h = fb_h<S, LAP>(s, zp, snp, csp);
        if (s > 0) h *= (LAP && s == S - 1) ? bhl : bht;
        lds_put4<4, ZPLANE>(H + s * ZSET + col, h[0], h[1], h[2], h[3]);
        }
      }
      __syncthreads();
      FB_STAMP(sp + 2);
      // the propagation's first W^T fragment: its L2 latency runs under the dW MFMAs
      FragQ<4> wn = wsp_frag<4, NT>(wsl, L, 1, j, rt, 0, lane);
      // dW_j: wave (ra, cb) = (wave >> 1, wave & 1) owns row tiles 2 ra, 2 ra + 1 (A: z̄ column reads
      // of the point-major P sets) x column tiles 4 cb .. 4 cb + 3 (B: transpose reads of H) -- 6
      // fragment reads per 8 MFMA triples (a wave owning one row tile x all 8 column tiles: 9)
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int u = 2 * ch + (g >> 1);
        const bool live = u < S;
        const int p0 = 8 * (g & 1);
        FragQ<4> af[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const unsigned short* pa =
              P + (live ? u : 0) * ZSET + (p0 + (c >> 2)) * LDB + 16 * (2 * ra + i) + 4 * (c & 3);
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const v4s lo = ds_read_tr16(pa + q * ZPLANE);
            const v4s hi = ds_read_tr16(pa + q * ZPLANE + 4 * LDB);
            const u32x2 wl = __builtin_bit_cast(u32x2, lo), wh = __builtin_bit_cast(u32x2, hi);
            af[i].q[q] = live ? u32x4{wl[0], wl[1], wh[0], wh[1]} : u32x4{0u, 0u, 0u, 0u};
          }
        }
        // B: h_{j-1} rows 16 ct + c at the chunk's 8 points -- transpose reads as A; the next column
        // tile's fragment is issued before this one's MFMAs (its LDS latency runs under them)
        auto bfrag = [&](int q4) __attribute__((always_inline)) {
          FragQ<4> bf;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const unsigned short* pb =
                H + (live ? u : 0) * ZSET + (p0 + (c >> 2)) * LDB + 16 * (4 * cb + q4) + 4 * (c & 3);
            const v4s lo = ds_read_tr16(pb + q * ZPLANE);
            const v4s hi = ds_read_tr16(pb + q * ZPLANE + 4 * LDB);
            const u32x2 wl = __builtin_bit_cast(u32x2, lo), wh = __builtin_bit_cast(u32x2, hi);
            bf.q[q] = u32x4{wl[0], wl[1], wh[0], wh[1]};
          }
          return bf;
        };
        FragQ<4> bf = bfrag(0);
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          FragQ<4> bn;
          if (q4 < 3) bn = bfrag(q4 + 1);
#pragma unroll
          for (int i = 0; i < 2; ++i) dacc[j - 1][4 * i + q4] = mfma_q<4>(af[i], bf, dacc[j - 1][4 * i + q4]);
          X6_SCHED_FENCE();
          if (q4 < 3) bf = bn;
        }
      }
      FB_STAMP(sp + 3);
      if (tile == t1 - 1) {
        // the block's last tile: dW_j is final -- its partial (fragment order, power of two undone) leaves
        // now and drains under the remaining layers' sweep instead of as one burst after the loop (round 6)
        floatx4* out = reinterpret_cast<floatx4*>(dpart + ((long)(j - 1) * nb + blockIdx.x) * W * W);
        const float f = ldexpf(1.f, -E[j - 1]);
#pragma unroll
        for (int q = 0; q < NT; ++q) out[((2 * ra + q / 4) * NT + 4 * cb + q % 4) * 64 + lane] = dacc[j - 1][q] * f;
      }
      // propagation: h̄_{j-1}[m] = sum_n W_j[n][m] z̄_j[n] (A = 2^8 W^T fragments, B = P rows)
      floatx4 nh[S];
#pragma unroll
      for (int s = 0; s < S; ++s) nh[s] = floatx4{0.f, 0.f, 0.f, 0.f};
      // the next (K chunk, stream) B fragment is issued before this one's MFMAs
      FragQ<4> pb = lds_frag<4, ZPLANE>(P + c * LDB + 8 * g);
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const FragQ<4> wt = wn;
        if (kc + 1 < KC) wn = wsp_frag<4, NT>(wsl, L, 1, j, rt, kc + 1, lane);
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int nk = s + 1 < S ? kc : kc + 1, ns = s + 1 < S ? s + 1 : 0;
          FragQ<4> pn;
          if (nk < KC) pn = lds_frag<4, ZPLANE>(P + ns * ZSET + c * LDB + 32 * nk + 8 * g);
          nh[s] = mfma_q<4>(wt, pb, nh[s]);
          X6_SCHED_FENCE();
          if (nk < KC) pb = pn;
        }
      }
      const float zun = ldexpf(1.f, -e) / kF16WScale;
#pragma unroll
      for (int s = 0; s < S; ++s) hb[s] = (nh[s] * zun) * (s == 0 ? 1.f : ((LAP && s == S - 1) ? bhl : bht));
#pragma unroll
      for (int s = 0; s < S; ++s) zc[s] = zp[s];
      fb_sincos(zc[0], sn, cs);
      FB_STAMP(sp + 4);
    };
    if constexpr (L >= 5) bwd_layer(std::integral_constant<int, 5>{});
    if constexpr (L >= 4) bwd_layer(std::integral_constant<int, 4>{});
    if constexpr (L >= 3) bwd_layer(std::integral_constant<int, 3>{});
    if constexpr (L >= 2) bwd_layer(std::integral_constant<int, 2>{});
    bwd_layer(std::integral_constant<int, 1>{});

    // first layer (K = d_in: exact fp32 VALU): zc = z_0 streams, sn / cs of z_0
    sine_rev<S, LAP>(hb, zc, sn, cs);  // hb = z̄_0
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = sum16(hb[0][r]);
      if (c == 0) sacc[(long)W * din + n0 + r] += v;
    }
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) {
      if (kk >= din) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = hb[0][r] * xk[kk];
#pragma unroll
        for (int i = 0; i < NTAN; ++i)
          if (i == kk) v += hb[1 + i][r];
        v = sum16(v);
        if (c == 0) sacc[(long)(n0 + r) * din + kk] += v;
      }
    }
    FB_STAMP(31);
  }

  // ---- the block's partials: dW of every hidden layer in fragment order (one 1 KiB wave store per
  // accumulator, the accumulator's power of two undone; reduce_dw_kernel frag = 1 scatters the
  // sums) -- stored inside the last tile's sweep, layer by layer; a block without tiles stores its
  // zeros here -- then the compact row ----
  if (t1 == t0) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, ra = wave >> 1, cb = wave & 1;
#pragma unroll
    for (int jl = 0; jl < L; ++jl) {
      floatx4* out = reinterpret_cast<floatx4*>(dpart + ((long)jl * nb + blockIdx.x) * W * W);
#pragma unroll
      for (int q = 0; q < NT; ++q) out[((2 * ra + q / 4) * NT + 4 * cb + q % 4) * 64 + lane] = dacc[jl][q];
    }
  }
  __syncthreads();  // every owner lane's last compact update
  for (int i = threadIdx.x; i < Ps; i += 512) small[(long)blockIdx.x * Ps + i] = sacc0[i];
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
// Balanced persistent grid (round 6): the launch lasts ceil(tiles / CUs) tile-times whatever the block
// count, so take the FEWEST blocks that still need no more tiles each -- 16,708 points = 1,045 tiles:
// 209 blocks x 5 instead of 256 blocks of 4 or 5; the shard's 523 tiles: 175 x 3 instead of 256 x 2-3 --
// the same critical path with 18-32 % fewer per-CU dW partials written here and re-read by the sums
inline int fb_blocks(long tiles) {
  const long cus = device_cus();
  if (tiles <= cus) return (int)(tiles > 0 ? tiles : 1);
  const long per = (tiles + cus - 1) / cus;
  return (int)((tiles + per - 1) / per);
}

// workspace floats: dW partials [layer][block][W^2] | compact rows [block][Ps]
inline long fb_work_floats_impl(long tiles, int din, int dout, int L) {
  const long nb = fb_blocks(tiles);
  return (long)L * nb * 128 * 128 + nb * small_count(din, dout, L, 128);
}

// phases: 1 the reverse sweep, 2 the sums (with A.m: + the Adam update, insr_siren_jet_bwd_grad_adam),
// 3 both (the same work buffer between a 1 and a 2)
template <int S, bool LAP, int L, int ZR, bool SAVED>
int fb_bwd_t(const FbJobs& J, int din, int dout, const float* prm, float* work, float* grad, int accumulate,
             int phases, const AdamArgs& A, hipStream_t st) {
  constexpr int W = 128;
  const int tiles = J.tstart[J.njobs];
  if (tiles <= 0) return 0;
  const int nb = fb_blocks(tiles);
  const long Ps = small_count(din, dout, L, W);
  if (Ps > kFbSmallMax || dout < 1 || dout > 3 || din < 1 || din > 3) return INSR_EINVAL;
  float* dpart = work;
  float* small = dpart + (long)L * nb * W * W;
  constexpr size_t lds = FbGeo<S, L, ZR, SAVED>::BYTES;
  static_assert(lds <= 163840, "LDS");
  static const bool attr = ((void)hipFuncSetAttribute((const void*)jet_fb_x6<S, LAP, L, ZR, SAVED>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds), true);  // once per instantiation (thread-safe static init)
  (void)attr;
  if (phases & 1) {
    if constexpr (SAVED) {
      if (J.seeds.nt) {  // the seeded instantiation: its block's tiles must fit the LDS stage
        constexpr size_t lds_s = FbGeo<S, L, ZR, true, true>::BYTES;
        static_assert(lds_s <= 163840, "LDS");
        static const bool attr_s = ((void)hipFuncSetAttribute((const void*)jet_fb_x6<S, LAP, L, ZR, true, true>,
                                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_s),
                                    true);
        (void)attr_s;
        if ((tiles + nb - 1) / nb > kFbSeedTiles) return INSR_EINVAL;
        hipLaunchKernelGGL((jet_fb_x6<S, LAP, L, ZR, true, true>), dim3(nb), dim3(512), lds_s, st, J, din, dout, prm,
                           dpart, small, Ps, nb, tiles);
      } else {
        hipLaunchKernelGGL((jet_fb_x6<S, LAP, L, ZR, SAVED>), dim3(nb), dim3(512), lds, st, J, din, dout, prm, dpart,
                           small, Ps, nb, tiles);
      }
    } else {
      if (J.seeds.nt) return INSR_EINVAL;
      hipLaunchKernelGGL((jet_fb_x6<S, LAP, L, ZR, SAVED>), dim3(nb), dim3(512), lds, st, J, din, dout, prm, dpart,
                         small, Ps, nb, tiles);
    }
  }
  if (!(phases & 2)) return (int)hipGetLastError();
  const int grad16 = (((uintptr_t)(grad + hidden_off(din, W, 1))) & 15) == 0 ? 1 : 0;
  const int wq = (W * W / 4 + 63) / 64;
  const int rows_x = (int)((Ps + 63) / 64);
  hipLaunchKernelGGL(reduce_dw_kernel, dim3((unsigned)(wq > rows_x ? wq : rows_x), L + 1), dim3(512), 0, st, dpart, nb,
                     din, W, grad, accumulate, grad16, 1, L, small, nb, Ps, dout, 1, nb, A);
  return (int)hipGetLastError();
}

}  // namespace insr
