// jet_wave.hip -- "wave-tile" SIREN jet kernels: one wave owns 16 collocation points
// and ALL neurons x streams of them in VGPRs; a block is 4 waves = 64 points.
// Best when the batch fills the chip (>= ~128 blocks); see jet_split.hip for small
// batches.  Math and layout: jet_common.hpp.
#include "jet_common.hpp"

namespace insr {
// ---------------------------------------------------------------------------
// forward jet
// ---------------------------------------------------------------------------
template <int NT, int S, bool LAP>
__global__ __launch_bounds__(kThreads, 1) void jet_fwd_wave(
    const float* __restrict__ x, int N, int din, int dout, int L, const float* __restrict__ prm,
    float* __restrict__ y, float* __restrict__ dy, float* __restrict__ lap, float* __restrict__ act) {
  constexpr int W = 16 * NT, LDW = W + 8;
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int ntiles = gridDim.x * kWaves;
  const int tile = blockIdx.x * kWaves + wave;
  const int p = tile * 16 + c;
  const bool valid = p < N;

  float xv[3] = {0.f, 0.f, 0.f};
  for (int j = 0; j < din; ++j) xv[j] = valid ? x[(long)p * din + j] : 0.f;

  floatx4 h[NT][S];
  // ---- layer 0 (K = d_in: VALU) ----
  {
    const float* W0 = prm;
    const float* b0 = prm + (long)W * din;
#pragma unroll
    for (int rt = 0; rt < NT; ++rt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * rt + 4 * g + r;
        float z = b0[n];
        for (int j = 0; j < din; ++j) z = fmaf(W0[n * din + j], xv[j], z);
        h[rt][0][r] = z;
#pragma unroll
        for (int i = 0; i < NTAN; ++i) h[rt][1 + i][r] = W0[n * din + i];
        if constexpr (LAP) h[rt][S - 1][r] = 0.f;
      }
    }
    if (act) save_streams<NT, S>(act_base(act, 0, ntiles, tile, S, NT), h, lane);
    sine_jet<NT, S, LAP>(h);
  }
  // ---- hidden layers: MFMA, A = W (LDS), B = h (registers) ----
  for (int j = 1; j <= L; ++j) {
    const float* Wj = prm + hidden_off(din, W, j);
    const float* bj = Wj + (long)W * W;
    __syncthreads();
    for (int idx = threadIdx.x; idx < W * W / 4; idx += kThreads) {
      const int n = idx / (W / 4), m4 = idx % (W / 4);
      *reinterpret_cast<floatx4*>(lds + n * LDW + 4 * m4) =
          *reinterpret_cast<const floatx4*>(Wj + (long)n * W + 4 * m4);
    }
    __syncthreads();
    floatx4 acc[NT][S];
#pragma unroll
    for (int rt = 0; rt < NT; ++rt) {
      acc[rt][0] = *reinterpret_cast<const floatx4*>(bj + 16 * rt + 4 * g);
#pragma unroll
      for (int s = 1; s < S; ++s) acc[rt][s] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int rt = 0; rt < NT; ++rt) {
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) {
        const floatx4 wa = *reinterpret_cast<const floatx4*>(lds + (16 * rt + c) * LDW + 16 * kt + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int s = 0; s < S; ++s) acc[rt][s] = mfma4(wa[r], h[kt][s][r], acc[rt][s]);
      }
    }
    if (act) save_streams<NT, S>(act_base(act, j, ntiles, tile, S, NT), acc, lane);
    sine_jet<NT, S, LAP>(acc);
#pragma unroll
    for (int rt = 0; rt < NT; ++rt)
#pragma unroll
      for (int s = 0; s < S; ++s) h[rt][s] = acc[rt][s];
  }
  // ---- output layer (d_out <= 3 rows: VALU + cross-lane sum) ----
  const float* Wo = prm + out_off(din, W, L);
  const float* bo = Wo + (long)dout * W;
  for (int o = 0; o < dout; ++o) {
    float sv[S];
#pragma unroll
    for (int s = 0; s < S; ++s) sv[s] = 0.f;
#pragma unroll
    for (int rt = 0; rt < NT; ++rt) {
      const floatx4 w4 = *reinterpret_cast<const floatx4*>(Wo + (long)o * W + 16 * rt + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int s = 0; s < S; ++s) sv[s] = fmaf(w4[r], h[rt][s][r], sv[s]);
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      sv[s] += __shfl_xor(sv[s], 16);
      sv[s] += __shfl_xor(sv[s], 32);
    }
    if (g == 0 && valid) {
      y[(long)p * dout + o] = sv[0] + bo[o];
      if (dy)
        for (int i = 0; i < NTAN; ++i) dy[((long)p * dout + o) * din + i] = sv[1 + i];
      if constexpr (LAP) {
        if (lap) lap[(long)p * dout + o] = sv[S - 1];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward jet
// ---------------------------------------------------------------------------
template <int NT, int S, bool LAP>
__global__ __launch_bounds__(kThreads, 1) void jet_bwd_wave(
    const float* __restrict__ x, int N, int din, int dout, int L, const float* __restrict__ prm,
    const float* __restrict__ act, const float* __restrict__ gy, const float* __restrict__ gdy,
    const float* __restrict__ glap, float* __restrict__ part, long P) {
  constexpr int W = 16 * NT, LDW = W + 8;
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  constexpr int TPW = (NT * NT + kWaves - 1) / kWaves;  // dW tiles per wave
  extern __shared__ __attribute__((aligned(16))) float lds[];
  // LDS: region A = max(W x LDW [W^T], 2 x W x kLdp [zb | h planes]); then reduction scratch
  constexpr int kRegionA = (W * LDW > 2 * W * kLdp) ? W * LDW : 2 * W * kLdp;
  float* wt = lds;
  float* zbp = lds;
  float* hpp = lds + W * kLdp;
  float* red = lds + kRegionA;  // [kWaves][W * 3]

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int ntiles = gridDim.x * kWaves;
  const int tile = blockIdx.x * kWaves + wave;
  const int p = tile * 16 + c;
  const bool valid = p < N;
  const int pl = wave * 16 + c;  // point index inside the block
  float* mypart = part + (long)blockIdx.x * P;

  float xv[3] = {0.f, 0.f, 0.f};
  for (int j = 0; j < din; ++j) xv[j] = valid ? x[(long)p * din + j] : 0.f;
  // adjoints of the jet outputs for this lane's point: ga[s][o]
  float ga[S][3];
#pragma unroll
  for (int s = 0; s < S; ++s)
    for (int o = 0; o < 3; ++o) ga[s][o] = 0.f;
  if (valid) {
    for (int o = 0; o < dout; ++o) {
      if (gy) ga[0][o] = gy[(long)p * dout + o];
      if (gdy)
        for (int i = 0; i < NTAN; ++i) ga[1 + i][o] = gdy[((long)p * dout + o) * din + i];
      if constexpr (LAP) {
        if (glap) ga[S - 1][o] = glap[(long)p * dout + o];
      }
    }
  }

  // reduce a per-lane value over the block's 64 points into red[wave][slot]; caller syncs
  auto wave_sum_store = [&](float v, int slot) {
    v = sum16(v);
    if (c == 0) red[wave * (3 * W) + slot] = v;
  };

  // ---- output layer ----
  floatx4 sn[NT], cs[NT];
  const float* baseL = act_base(act, L, ntiles, tile, S, NT);
  load_z_sincos<NT>(baseL, S, lane, sn, cs);
  const float* Wo = prm + out_off(din, W, L);
  const long wo_off = out_off(din, W, L);
  {
    // dW_out[o][n] = sum_p sum_s ga[s][o] * h_s[n][p]
    for (int o = 0; o < dout; ++o) {
#pragma unroll
      for (int rt = 0; rt < NT; ++rt) {
        floatx4 acc4 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const floatx4 hs = h_stream<NT, S, LAP>(baseL, s, rt, lane, sn[rt], cs[rt]);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc4[r] = fmaf(ga[s][o], hs[r], acc4[r]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) wave_sum_store(acc4[r], o * W + 16 * rt + 4 * g + r);
      }
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < dout * W; idx += kThreads)
      mypart[wo_off + idx] = red[idx] + red[3 * W + idx] + red[6 * W + idx] + red[9 * W + idx];
    __syncthreads();
    // bias: every wave sums its 16 points (lanes g==0 hold distinct points)
    for (int o = 0; o < dout; ++o) {
      float v = (g == 0) ? ga[0][o] : 0.f;
      v = sum16(v);
      if (lane == 0) red[wave * (3 * W) + o] = v;
    }
    __syncthreads();
    if (threadIdx.x < dout)
      mypart[wo_off + (long)dout * W + threadIdx.x] =
          red[threadIdx.x] + red[3 * W + threadIdx.x] + red[6 * W + threadIdx.x] + red[9 * W + threadIdx.x];
  }
  // hb_L[s][n] = sum_o Wo[o][n] * ga[s][o]
  floatx4 hb[NT][S];
#pragma unroll
  for (int rt = 0; rt < NT; ++rt)
#pragma unroll
    for (int s = 0; s < S; ++s) hb[rt][s] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int o = 0; o < dout; ++o) {
#pragma unroll
    for (int rt = 0; rt < NT; ++rt) {
      const floatx4 w4 = *reinterpret_cast<const floatx4*>(Wo + (long)o * W + 16 * rt + 4 * g);
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int r = 0; r < 4; ++r) hb[rt][s][r] = fmaf(w4[r], ga[s][o], hb[rt][s][r]);
    }
  }

  // ---- sine layers j = L .. 0 ----
  for (int j = L; j >= 0; --j) {
    const float* basej = act_base(act, j, ntiles, tile, S, NT);
    // (1) sine reverse: hb -> zb (in place), using cached sin/cos of z_j
#pragma unroll
    for (int rt = 0; rt < NT; ++rt) {
      floatx4 zs[S];
#pragma unroll
      for (int s = 0; s < S; ++s)
        zs[s] = (s == 0) ? floatx4{0.f, 0.f, 0.f, 0.f}
                         : *reinterpret_cast<const floatx4*>(basej + ((s * NT + rt) * 64 + lane) * 4);
      sine_rev<S, LAP>(hb[rt], zs, sn[rt], cs[rt]);
    }
    const long boff = (j == 0) ? (long)W * din : hidden_off(din, W, j) + (long)W * W;
    // (2) bias gradient: sum over points of zb_value
    __syncthreads();
#pragma unroll
    for (int rt = 0; rt < NT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) wave_sum_store(valid ? hb[rt][0][r] : 0.f, 16 * rt + 4 * g + r);
    __syncthreads();
    for (int idx = threadIdx.x; idx < W; idx += kThreads)
      mypart[boff + idx] = red[idx] + red[3 * W + idx] + red[6 * W + idx] + red[9 * W + idx];

    if (j == 0) {
      // dW0[n][i] = sum_p zb[n][p] x_i[p] + tb_i[n][p]
      __syncthreads();
      for (int i = 0; i < din; ++i) {
#pragma unroll
        for (int rt = 0; rt < NT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = hb[rt][0][r] * xv[i];
            if (i < NTAN) v += hb[rt][1 + i][r];
            wave_sum_store(valid ? v : 0.f, i * W + 16 * rt + 4 * g + r);
          }
      }
      __syncthreads();
      for (int idx = threadIdx.x; idx < W * din; idx += kThreads) {
        const int n = idx / din, i = idx % din;
        const int slot = i * W + n;
        mypart[(long)n * din + i] = red[slot] + red[3 * W + slot] + red[6 * W + slot] + red[9 * W + slot];
      }
      break;
    }

    // (3) sin/cos of z_{j-1} (needed for h_{j-1} now and the sine reverse next)
    const float* basep = act_base(act, j - 1, ntiles, tile, S, NT);
    load_z_sincos<NT>(basep, S, lane, sn, cs);

    // (4) dW_j = sum_s Zb_s (W x 64pts) . H_{j-1,s}^T (64pts x W), via LDS planes
    floatx4 dacc[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) dacc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < S; ++s) {
      __syncthreads();
#pragma unroll
      for (int rt = 0; rt < NT; ++rt) {
        const floatx4 hs = h_stream<NT, S, LAP>(basep, s, rt, lane, sn[rt], cs[rt]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 16 * rt + 4 * g + r;
          zbp[n * kLdp + pl] = valid ? hb[rt][s][r] : 0.f;
          hpp[n * kLdp + pl] = hs[r];
        }
      }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const int tt = wave * TPW + t;
        if (tt < NT * NT) {
          const int rt = tt / NT, ct = tt % NT;
#pragma unroll
          for (int v = 0; v < kPts / 16; ++v) {
            const floatx4 a4 = *reinterpret_cast<const floatx4*>(zbp + (16 * rt + c) * kLdp + 16 * v + 4 * g);
            const floatx4 b4 = *reinterpret_cast<const floatx4*>(hpp + (16 * ct + c) * kLdp + 16 * v + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) dacc[t] = mfma4(a4[r], b4[r], dacc[t]);
          }
        }
      }
    }
    {
      float* dW = mypart + hidden_off(din, W, j);
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const int tt = wave * TPW + t;
        if (tt < NT * NT) {
          const int rt = tt / NT, ct = tt % NT;
#pragma unroll
          for (int r = 0; r < 4; ++r) dW[(long)(16 * rt + 4 * g + r) * W + 16 * ct + c] = dacc[t][r];
        }
      }
    }
    // (5) propagate: hb_{j-1} = W_j^T zb   (A = W^T staged in LDS, B = zb in registers)
    const float* Wj = prm + hidden_off(din, W, j);
    __syncthreads();
    for (int idx = threadIdx.x; idx < W * W / 4; idx += kThreads) {
      const int n = idx / (W / 4), m4 = idx % (W / 4);
      const floatx4 v = *reinterpret_cast<const floatx4*>(Wj + (long)n * W + 4 * m4);
#pragma unroll
      for (int r = 0; r < 4; ++r) wt[(4 * m4 + r) * LDW + n] = v[r];
    }
    __syncthreads();
    floatx4 nh[NT][S];
#pragma unroll
    for (int rt = 0; rt < NT; ++rt)
#pragma unroll
      for (int s = 0; s < S; ++s) nh[rt][s] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int rt = 0; rt < NT; ++rt) {
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) {
        const floatx4 wa = *reinterpret_cast<const floatx4*>(wt + (16 * rt + c) * LDW + 16 * kt + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int s = 0; s < S; ++s) nh[rt][s] = mfma4(wa[r], hb[kt][s][r], nh[rt][s]);
      }
    }
#pragma unroll
    for (int rt = 0; rt < NT; ++rt)
#pragma unroll
      for (int s = 0; s < S; ++s) hb[rt][s] = nh[rt][s];
  }
}

static size_t fwd_lds(int NT) { return (size_t)(16 * NT) * (16 * NT + 8) * sizeof(float); }
static size_t bwd_lds(int NT) {
  const int W = 16 * NT, LDW = W + 8;
  const size_t a = (size_t)((W * LDW > 2 * W * kLdp) ? W * LDW : 2 * W * kLdp);
  return (a + (size_t)kWaves * 3 * W) * sizeof(float);
}

template <int NT, int S, bool LAP>
int launch_fwd(const float* x, int N, int din, int dout, int L, const float* prm, float* y, float* dy, float* lap,
               float* act, hipStream_t st) {
  const int nb = (N + kPts - 1) / kPts;
  const size_t lds = fwd_lds(NT);
  static bool attr_set = false;  // once per instantiation (not a stream op: capture-safe)
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)jet_fwd_wave<NT, S, LAP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((jet_fwd_wave<NT, S, LAP>), dim3(nb), dim3(kThreads), lds, st, x, N, din, dout, L, prm, y,
                     dy, lap, act);
  return (int)hipGetLastError();
}

template <int NT, int S, bool LAP>
int launch_bwd(const float* x, int N, int din, int dout, int L, const float* prm, const float* act,
               const float* gy, const float* gdy, const float* glap, float* part, long P, hipStream_t st) {
  const int nb = (N + kPts - 1) / kPts;
  const size_t lds = bwd_lds(NT);
  static bool attr_set = false;  // once per instantiation (not a stream op: capture-safe)
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)jet_bwd_wave<NT, S, LAP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((jet_bwd_wave<NT, S, LAP>), dim3(nb), dim3(kThreads), lds, st, x, N, din, dout, L, prm,
                     act, gy, gdy, glap, part, P);
  return (int)hipGetLastError();
}

int dispatch_fwd_wave(int NT, int S, bool LAP, const float* x, int N, int din, int dout, int L, const float* prm,
                 float* y, float* dy, float* lap, float* act, hipStream_t st) {
  switch (NT) {
    case 2: INSR_DISPATCH(2, launch_fwd, x, N, din, dout, L, prm, y, dy, lap, act, st)
    case 4: INSR_DISPATCH(4, launch_fwd, x, N, din, dout, L, prm, y, dy, lap, act, st)
    case 8: INSR_DISPATCH(8, launch_fwd, x, N, din, dout, L, prm, y, dy, lap, act, st)
    default: return INSR_EWIDTH;
  }
}

int dispatch_bwd_wave(int NT, int S, bool LAP, const float* x, int N, int din, int dout, int L, const float* prm,
                 const float* act, const float* gy, const float* gdy, const float* glap, float* part, long P,
                 hipStream_t st) {
  switch (NT) {
    case 2: INSR_DISPATCH(2, launch_bwd, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    case 4: INSR_DISPATCH(4, launch_bwd, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    case 8: INSR_DISPATCH(8, launch_bwd, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    default: return INSR_EWIDTH;
  }
}


}  // namespace insr
