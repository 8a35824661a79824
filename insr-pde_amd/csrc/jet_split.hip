// jet_split.hip -- "tile-split" SIREN jet kernels for SMALL batches (boundary bands,
// fixed-point constraints, advection with few samples).
//
// A wave-tile kernel (jet_wave.hip) gives each 16-point tile to ONE wave; with a
// few hundred points that is a handful of blocks and the run time is one wave's
// serial chain through every layer.  Here a 16-point tile is one block of 4 waves
// and the OUTPUT NEURONS of every layer are split over the waves (wave w owns row
// tiles w, w+4, ...), so each wave's chain per layer is ~1/4 as long.  Layers
// exchange activations through LDS (point-major [stream][point][neuron], read as
// the B operand with ds_read_b128); each wave streams its slice of W straight
// from L2 into the A operand.  The backward transposes the sine-reverse adjoints
// through LDS once per layer for both GEMMs (dW and the W^T propagation).
//
// Saved activations use exactly the wave-tile layout (jet_common.hpp), one
// partial-gradient row is written per 16-point tile.
#include "jet_common.hpp"

namespace insr {

constexpr int kSplitWaves = 4;

template <int NT>
struct SplitGeo {
  static constexpr int W = 16 * NT;
  static constexpr int RPW = (NT + kSplitWaves - 1) / kSplitWaves;  // row tiles per wave
  static constexpr int LDH = W + 8;                                  // point-major rows [p][W]
};

template <int NT, int S>
__device__ __forceinline__ void store_point_major(float* buf, const floatx4 (&a)[SplitGeo<NT>::RPW][S], int wave,
                                                  int g, int c) {
  constexpr int LDH = SplitGeo<NT>::LDH;
#pragma unroll
  for (int i = 0; i < SplitGeo<NT>::RPW; ++i) {
    const int rt = wave + kSplitWaves * i;
    if (rt < NT) {
#pragma unroll
      for (int s = 0; s < S; ++s) *reinterpret_cast<floatx4*>(buf + (s * 16 + c) * LDH + 16 * rt + 4 * g) = a[i][s];
    }
  }
}

template <int NT, int S, bool LAP>
__global__ __launch_bounds__(256) void jet_fwd_split(const float* __restrict__ x, int N, int din, int dout, int L,
                                                     const float* __restrict__ prm, float* __restrict__ y,
                                                     float* __restrict__ dy, float* __restrict__ lap,
                                                     float* __restrict__ act) {
  using G = SplitGeo<NT>;
  constexpr int W = G::W, RPW = G::RPW, LDH = G::LDH;
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int kBuf = S * 16 * LDH;    // one activation buffer; two ping-pong
  float* red = lds + 2 * kBuf;          // [wave][S][3][16]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int tile = blockIdx.x, ntiles = ((N + 63) / 64) * 4;  // same act layout as jet_wave.hip
  const int p = tile * 16 + c;
  const bool valid = p < N;
  float xv[3] = {0.f, 0.f, 0.f};
  for (int j = 0; j < din; ++j) xv[j] = valid ? x[(long)p * din + j] : 0.f;

  floatx4 a[RPW][S];
  {  // layer 0 (VALU)
    const float* W0 = prm;
    const float* b0 = prm + (long)W * din;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int rt = wave + kSplitWaves * i;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float z = 0.f;
        if (rt < NT) {
          const int n = 16 * rt + 4 * g + r;
          z = b0[n];
          for (int j = 0; j < din; ++j) z = fmaf(W0[n * din + j], xv[j], z);
#pragma unroll
          for (int t = 0; t < NTAN; ++t) a[i][1 + t][r] = W0[n * din + t];
        } else {
#pragma unroll
          for (int t = 0; t < NTAN; ++t) a[i][1 + t][r] = 0.f;
        }
        a[i][0][r] = z;
        if constexpr (LAP) a[i][S - 1][r] = 0.f;
      }
    }
    if (act) {
      float* base = act_base(act, 0, ntiles, tile, S, NT);
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        const int rt = wave + kSplitWaves * i;
        if (rt < NT)
#pragma unroll
          for (int s = 0; s < S; ++s)
            *reinterpret_cast<floatx4*>(base + ((s * NT + rt) * 64 + lane) * 4) = a[i][s];
      }
    }
    sine_jet<RPW, S, LAP>(a);
    store_point_major<NT, S>(lds, a, wave, g, c);
    __syncthreads();
  }
  for (int j = 1; j <= L; ++j) {
    const float* hin = lds + ((j - 1) & 1) * kBuf;
    float* hout = lds + (j & 1) * kBuf;
    const float* Wj = prm + hidden_off(din, W, j);
    const float* bj = Wj + (long)W * W;
    floatx4 wr[RPW][NT];
    floatx4 acc[RPW][S];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int rt = wave + kSplitWaves * i;
      const int rrow = rt < NT ? rt : 0;
#pragma unroll
      for (int kt = 0; kt < NT; ++kt)
        wr[i][kt] = *reinterpret_cast<const floatx4*>(Wj + (long)(16 * rrow + c) * W + 16 * kt + 4 * g);
      acc[i][0] = *reinterpret_cast<const floatx4*>(bj + 16 * rrow + 4 * g);
#pragma unroll
      for (int s = 1; s < S; ++s) acc[i][s] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const floatx4 hv = *reinterpret_cast<const floatx4*>(hin + (s * 16 + c) * LDH + 16 * kt + 4 * g);
#pragma unroll
        for (int i = 0; i < RPW; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][s] = mfma4(wr[i][kt][r], hv[r], acc[i][s]);
      }
    }
    if (act) {
      float* base = act_base(act, j, ntiles, tile, S, NT);
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        const int rt = wave + kSplitWaves * i;
        if (rt < NT)
#pragma unroll
          for (int s = 0; s < S; ++s)
            *reinterpret_cast<floatx4*>(base + ((s * NT + rt) * 64 + lane) * 4) = acc[i][s];
      }
    }
    sine_jet<RPW, S, LAP>(acc);
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int s = 0; s < S; ++s) a[i][s] = acc[i][s];
    store_point_major<NT, S>(hout, a, wave, g, c);
    __syncthreads();
  }
  // output layer: each wave sums its own neurons, waves combine through LDS
  const float* Wo = prm + out_off(din, W, L);
  const float* bo = Wo + (long)dout * W;
  for (int o = 0; o < dout; ++o) {
    float sv[S];
#pragma unroll
    for (int s = 0; s < S; ++s) sv[s] = 0.f;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int rt = wave + kSplitWaves * i;
      if (rt < NT) {
        const floatx4 w4 = *reinterpret_cast<const floatx4*>(Wo + (long)o * W + 16 * rt + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int s = 0; s < S; ++s) sv[s] = fmaf(w4[r], a[i][s][r], sv[s]);
      }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      sv[s] += __shfl_xor(sv[s], 16);
      sv[s] += __shfl_xor(sv[s], 32);
      if (g == 0) red[((wave * S + s) * 3 + o) * 16 + c] = sv[s];
    }
  }
  __syncthreads();
  if (wave == 0 && g == 0 && valid) {
    for (int o = 0; o < dout; ++o) {
      float tot[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        tot[s] = 0.f;
        for (int w = 0; w < kSplitWaves; ++w) tot[s] += red[((w * S + s) * 3 + o) * 16 + c];
      }
      y[(long)p * dout + o] = tot[0] + bo[o];
      if (dy)
        for (int t = 0; t < NTAN; ++t) dy[((long)p * dout + o) * din + t] = tot[1 + t];
      if constexpr (LAP) {
        if (lap) lap[(long)p * dout + o] = tot[S - 1];
      }
    }
  }
}

template <int NT, int S, bool LAP>
__global__ __launch_bounds__(256) void jet_bwd_split(const float* __restrict__ x, int N, int din, int dout, int L,
                                                     const float* __restrict__ prm, const float* __restrict__ act,
                                                     const float* __restrict__ gy, const float* __restrict__ gdy,
                                                     const float* __restrict__ glap, float* __restrict__ part,
                                                     long P) {
  using G = SplitGeo<NT>;
  constexpr int W = G::W, RPW = G::RPW, LDH = G::LDH;
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  // Both planes point-major [S][16 points][LDH]: zbp is read as b128 rows for the
  // propagation B operand and as 4 b32 columns for the dW A operand; hpp likewise
  // for the dW B operand.  2 x S x 16 x LDH floats (70 KB at S=4, W=128): two
  // blocks fit one CU.
  float* zbp = lds;                       // zb of layer j
  float* hpp = lds + S * 16 * LDH;        // h of layer j-1
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int tile = blockIdx.x, ntiles = ((N + 63) / 64) * 4;  // same act layout as jet_wave.hip
  const int p = tile * 16 + c;
  const bool valid = p < N;
  float* mypart = part + (long)tile * P;
  float xv[3] = {0.f, 0.f, 0.f};
  for (int j = 0; j < din; ++j) xv[j] = valid ? x[(long)p * din + j] : 0.f;
  float ga[S][3];
#pragma unroll
  for (int s = 0; s < S; ++s)
    for (int o = 0; o < 3; ++o) ga[s][o] = 0.f;
  if (valid) {
    for (int o = 0; o < dout; ++o) {
      if (gy) ga[0][o] = gy[(long)p * dout + o];
      if (gdy)
        for (int t = 0; t < NTAN; ++t) ga[1 + t][o] = gdy[((long)p * dout + o) * din + t];
      if constexpr (LAP) {
        if (glap) ga[S - 1][o] = glap[(long)p * dout + o];
      }
    }
  }

  floatx4 sn[RPW], cs[RPW];
  auto load_sc = [&](const float* base, floatx4 (&s_)[RPW], floatx4 (&c_)[RPW]) {
    floatx4 z[RPW];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int rt = wave + kSplitWaves * i;
      z[i] = rt < NT ? *reinterpret_cast<const floatx4*>(base + (rt * 64 + lane) * 4) : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) amax = fmaxf(amax, fabsf(OMEGA * z[i][r]));
    }
    const bool big = wave_any_big(amax);
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float a_, b_;
        if (big)
          sincosf(OMEGA * z[i][r], &a_, &b_);
        else
          sincos_fast(OMEGA * z[i][r], a_, b_);
        s_[i][r] = a_;
        c_[i][r] = b_;
      }
  };

  // ---- output layer ----
  const float* baseL = act_base(act, L, ntiles, tile, S, NT);
  load_sc(baseL, sn, cs);
  const float* Wo = prm + out_off(din, W, L);
  const long wo_off = out_off(din, W, L);
  floatx4 hb[RPW][S];
#pragma unroll
  for (int i = 0; i < RPW; ++i)
#pragma unroll
    for (int s = 0; s < S; ++s) hb[i][s] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int o = 0; o < dout; ++o) {
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int rt = wave + kSplitWaves * i;
      if (rt >= NT) continue;
      floatx4 acc4 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const floatx4 hs = h_stream<NT, S, LAP>(baseL, s, rt, lane, sn[i], cs[i]);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc4[r] = fmaf(ga[s][o], hs[r], acc4[r]);
      }
      const floatx4 w4 = *reinterpret_cast<const floatx4*>(Wo + (long)o * W + 16 * rt + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = sum16(acc4[r]);
        if (c == 0) mypart[wo_off + (long)o * W + 16 * rt + 4 * g + r] = v;
#pragma unroll
        for (int s = 0; s < S; ++s) hb[i][s][r] = fmaf(w4[r], ga[s][o], hb[i][s][r]);
      }
    }
    if (wave == 0) {  // db_out[o]: each point counted once (lanes g == 0)
      const float v = sum16(g == 0 ? ga[0][o] : 0.f);
      if (lane == 0) mypart[wo_off + (long)dout * W + o] = v;
    }
  }

  // ---- sine layers j = L .. 0 ----
  for (int j = L; j >= 0; --j) {
    const float* basej = act_base(act, j, ntiles, tile, S, NT);
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int rt = wave + kSplitWaves * i;
      floatx4 zs[S];
#pragma unroll
      for (int s = 0; s < S; ++s)
        zs[s] = (s == 0 || rt >= NT)
                    ? floatx4{0.f, 0.f, 0.f, 0.f}
                    : *reinterpret_cast<const floatx4*>(basej + ((s * NT + rt) * 64 + lane) * 4);
      sine_rev<S, LAP>(hb[i], zs, sn[i], cs[i]);
    }
    const long boff = (j == 0) ? (long)W * din : hidden_off(din, W, j) + (long)W * W;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int rt = wave + kSplitWaves * i;
      if (rt >= NT) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = sum16(hb[i][0][r]);
        if (c == 0) mypart[boff + 16 * rt + 4 * g + r] = v;
      }
    }
    if (j == 0) {
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        const int rt = wave + kSplitWaves * i;
        if (rt >= NT) continue;
        for (int t = 0; t < din; ++t) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = hb[i][0][r] * xv[t];
            if (t < NTAN) v += hb[i][1 + t][r];
            v = sum16(v);
            if (c == 0) mypart[(long)(16 * rt + 4 * g + r) * din + t] = v;
          }
        }
      }
      break;
    }
    // sin/cos of z_{j-1}: h_{j-1} now, and the sine reverse of the next iteration
    const float* basep = act_base(act, j - 1, ntiles, tile, S, NT);
    floatx4 snp[RPW], csp[RPW];
    load_sc(basep, snp, csp);
    __syncthreads();  // previous iteration's LDS readers are done
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int rt = wave + kSplitWaves * i;
      if (rt >= NT) continue;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const floatx4 hs = h_stream<NT, S, LAP>(basep, s, rt, lane, snp[i], csp[i]);
        *reinterpret_cast<floatx4*>(zbp + (s * 16 + c) * LDH + 16 * rt + 4 * g) = hb[i][s];
        *reinterpret_cast<floatx4*>(hpp + (s * 16 + c) * LDH + 16 * rt + 4 * g) = hs;
      }
    }
    __syncthreads();
    // dW_j rows of my tiles: K = 16 points x S streams
    {
      float* dW = mypart + hidden_off(din, W, j);
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        const int rt = wave + kSplitWaves * i;
        if (rt >= NT) continue;
        floatx4 dacc[NT];
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) dacc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < S; ++s) {
          // k = point 4g + r: A[n = 16rt + c][k], B[k][m = 16ct + c] as column reads
          floatx4 a4;
#pragma unroll
          for (int r = 0; r < 4; ++r) a4[r] = zbp[(s * 16 + 4 * g + r) * LDH + 16 * rt + c];
#pragma unroll
          for (int ct = 0; ct < NT; ++ct) {
#pragma unroll
            for (int r = 0; r < 4; ++r) dacc[ct] = mfma4(a4[r], hpp[(s * 16 + 4 * g + r) * LDH + 16 * ct + c], dacc[ct]);
          }
        }
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r) dW[(long)(16 * rt + 4 * g + r) * W + 16 * ct + c] = dacc[ct][r];
      }
    }
    // propagate: hb_{j-1}[m] (my tiles) = sum_n W_j[n][m] zb[n]; A = W^T from L2, B = zb from LDS
    {
      const float* Wj = prm + hidden_off(din, W, j);
      floatx4 nh[RPW][S];
#pragma unroll
      for (int i = 0; i < RPW; ++i)
#pragma unroll
        for (int s = 0; s < S; ++s) nh[i][s] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) {
        floatx4 wa[RPW];
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
          const int rt = wave + kSplitWaves * i;
          const int m = 16 * (rt < NT ? rt : 0) + c;
#pragma unroll
          for (int r = 0; r < 4; ++r) wa[i][r] = Wj[(long)(16 * kt + 4 * g + r) * W + m];
        }
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const floatx4 b4 = *reinterpret_cast<const floatx4*>(zbp + (s * 16 + c) * LDH + 16 * kt + 4 * g);
#pragma unroll
          for (int i = 0; i < RPW; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) nh[i][s] = mfma4(wa[i][r], b4[r], nh[i][s]);
        }
      }
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        sn[i] = snp[i];
        cs[i] = csp[i];
#pragma unroll
        for (int s = 0; s < S; ++s) hb[i][s] = nh[i][s];
      }
    }
  }
}

static size_t fwd_split_lds(int NT, int S) {
  const int W = 16 * NT, LDH = W + 8;
  return ((size_t)2 * S * 16 * LDH + (size_t)kSplitWaves * S * 3 * 16) * sizeof(float);
}
static size_t bwd_split_lds(int NT, int S) {
  const int W = 16 * NT, LDH = W + 8;
  return (size_t)2 * S * 16 * LDH * sizeof(float);
}

template <int NT, int S, bool LAP>
int launch_fwd_split(const float* x, int N, int din, int dout, int L, const float* prm, float* y, float* dy,
                     float* lap, float* act, hipStream_t st) {
  const int nb = (N + 15) / 16;
  const size_t lds = fwd_split_lds(NT, S);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)jet_fwd_split<NT, S, LAP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((jet_fwd_split<NT, S, LAP>), dim3(nb), dim3(256), lds, st, x, N, din, dout, L, prm, y, dy,
                     lap, act);
  return (int)hipGetLastError();
}

template <int NT, int S, bool LAP>
int launch_bwd_split(const float* x, int N, int din, int dout, int L, const float* prm, const float* act,
                     const float* gy, const float* gdy, const float* glap, float* part, long P, hipStream_t st) {
  const int nb = (N + 15) / 16;
  const size_t lds = bwd_split_lds(NT, S);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)jet_bwd_split<NT, S, LAP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((jet_bwd_split<NT, S, LAP>), dim3(nb), dim3(256), lds, st, x, N, din, dout, L, prm, act, gy,
                     gdy, glap, part, P);
  return (int)hipGetLastError();
}

int dispatch_fwd_split(int NT, int S, bool LAP, const float* x, int N, int din, int dout, int L, const float* prm,
                       float* y, float* dy, float* lap, float* act, hipStream_t st) {
  switch (NT) {
    case 2: INSR_DISPATCH(2, launch_fwd_split, x, N, din, dout, L, prm, y, dy, lap, act, st)
    case 4: INSR_DISPATCH(4, launch_fwd_split, x, N, din, dout, L, prm, y, dy, lap, act, st)
    case 8: INSR_DISPATCH(8, launch_fwd_split, x, N, din, dout, L, prm, y, dy, lap, act, st)
    default: return INSR_EWIDTH;
  }
}

int dispatch_bwd_split(int NT, int S, bool LAP, const float* x, int N, int din, int dout, int L, const float* prm,
                       const float* act, const float* gy, const float* gdy, const float* glap, float* part, long P,
                       hipStream_t st) {
  switch (NT) {
    case 2: INSR_DISPATCH(2, launch_bwd_split, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    case 4: INSR_DISPATCH(4, launch_bwd_split, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    case 8: INSR_DISPATCH(8, launch_bwd_split, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    default: return INSR_EWIDTH;
  }
}

}  // namespace insr
