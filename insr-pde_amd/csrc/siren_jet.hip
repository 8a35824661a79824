// siren_jet.hip -- fused SIREN Taylor-jet forward/backward for gfx950 (MI355X, CDNA4).
//
// Replaces, for the INSR-PDE per-iteration training loop, the aten graph that
// the reference builds with torch.autograd (create_graph=True):
//   MLP.forward ............................ base/networks.py:25-27,67-71
//   gradient / divergence / jacobian ....... base/diff_ops.py:44-82
//   laplace = divergence(gradient) ......... base/diff_ops.py:33-41
//   loss.backward() to the parameters ..... base/baseModel.py:73-78
//
// Math.  Linear layer k: z = W_k h + b_k.  Sine layer: h = sin(w z), w = 30.
// A forward Taylor jet carries, per point and neuron, S streams:
//   value z, tangents t_i = dz/dx_i (i < d), optionally q = sum_i d2z/dx_i^2.
// Linear layers act on every stream with the same W (bias on the value only),
// so a layer is ONE GEMM over (streams x points).  The sine couples streams
// per (point, neuron), lane-locally:
//   h = s,  dh_i = w c t_i,  ddh = w c q - w^2 s sum_i t_i^2       (s,c = sin,cos(w z))
// and its reverse (adjoints hb, dhb_i, ddhb -> zb, tb_i, qb):
//   zb  = w c hb - w^2 s sum_i t_i dhb_i - ddhb (w^2 s q + w^3 c sum_i t_i^2)
//   tb_i = w c dhb_i - 2 w^2 s t_i ddhb,   qb = w c ddhb
// Weight gradients: dW_k = sum_{streams,points} zb_stream (x) h_prev_stream.
//
// Layout on the chip ("transposed" orientation, MFMA v_mfma_f32_16x16x4_f32,
// exact fp32 = the fp32 matrix rate, no xf32 on gfx950):
//   * a wave owns 16 points = the 16 MFMA columns; neurons are MFMA rows.
//   * activations of all W neurons x S streams live in VGPRs as floatx4
//     h[rt][s] (rows 16rt+4g+r, column = point lane&15), which is exactly the
//     MFMA C/D layout AND the B-operand layout of the next layer, so layers
//     chain in registers with no LDS round trip.
//   * weights are the A operand, staged once per layer per block into LDS
//     (row stride W+8 floats: conflict-free ds_read_b128).
//   * the forward saves pre-activation streams to HBM in the MFMA-native
//     layout (each store = one contiguous 1 KiB wave write).
//   * the backward rebuilds sin/cos from the saved z, runs the sine reverse
//     lane-locally, and computes dW as an MFMA GEMM over the block's 64
//     points (operands transposed through LDS), writing one partial gradient
//     per block; insr_reduce_partials sums them in a fixed order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/insr_siren.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define OMEGA 30.0f
#define OMEGA2 900.0f
#define OMEGA3 27000.0f

namespace {

constexpr int kThreads = 256;  // 4 waves
constexpr int kWaves = 4;
constexpr int kPts = 64;       // points per block (16 per wave)
constexpr int kLdp = kPts + 8; // padded row of the point-major LDS planes

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__host__ __device__ __forceinline__ long hidden_off(int din, int W, int j) {
  // offset of net.{2j}.weight for hidden linear j >= 1
  return (long)W * din + W + (long)(j - 1) * ((long)W * W + W);
}
__host__ __device__ __forceinline__ long out_off(int din, int W, int L) {
  return (long)W * din + W + (long)L * ((long)W * W + W);
}

// wave-tile base of layer `layer` in the saved-activation buffer
__device__ __forceinline__ float* act_base(float* act, int layer, int ntiles, int tile, int S, int NT) {
  return act + ((long)layer * ntiles + tile) * (long)(S * NT) * 256;
}
__device__ __forceinline__ const float* act_base(const float* act, int layer, int ntiles, int tile, int S,
                                                 int NT) {
  return act + ((long)layer * ntiles + tile) * (long)(S * NT) * 256;
}

// sum over the 16 point-lanes that share lane>>4
__device__ __forceinline__ float sum16(float v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  return v;
}

// ---------------------------------------------------------------------------
// sin / cos of w*z.  Straight-line Cody-Waite reduction by pi/2 (3-part constant,
// valid for |x| <= 8192) + minimax polynomials on [-pi/4, pi/4]: ~1 ulp, ~20 VALU
// ops for the pair, no branches, so the compiler can interleave it with MFMAs.
// A wave with any |x| > 8192 takes the libm (ocml) path instead (uniform branch).
// ---------------------------------------------------------------------------
constexpr float kFastArgMax = 8192.0f;

__device__ __forceinline__ void sincos_fast(float x, float& s, float& c) {
  const float n = rintf(x * 0.636619772367581343f);
  float r = fmaf(-n, 1.5703125f, x);
  r = fmaf(-n, 4.837512969970703125e-4f, r);
  r = fmaf(-n, 7.54978995489188216e-8f, r);
  const float z = r * r;
  const float ps = fmaf(r * z, fmaf(z, fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f), -1.6666654611e-1f), r);
  const float pc = fmaf(z * z, fmaf(z, fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f),
                                    4.166664568298827e-2f), fmaf(-0.5f, z, 1.0f));
  const int q = (int)n;
  const float a = (q & 1) ? pc : ps;   // |sin|
  const float b = (q & 1) ? ps : pc;   // |cos|
  s = (q & 2) ? -a : a;
  c = ((q + 1) & 2) ? -b : b;
}

__device__ __forceinline__ float sin_fast(float x) {
  float s, c;
  sincos_fast(x, s, c);
  return s;
}

// true if any lane of the wave holds an argument outside the fast range
__device__ __forceinline__ bool wave_any_big(float amax) {
  return __any(amax > kFastArgMax);
}

// ---------------------------------------------------------------------------
// forward jet
// ---------------------------------------------------------------------------
template <int NT, int S, bool LAP, bool FAST>
__device__ __forceinline__ void sine_jet_impl(floatx4 (&a)[NT][S]) {
  constexpr int NTAN = LAP ? S - 2 : S - 1;
#pragma unroll
  for (int rt = 0; rt < NT; ++rt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float arg = OMEGA * a[rt][0][r];
      float sn, cs;
      if constexpr (S == 1) {  // value-only jet: sin is all we need
        if constexpr (FAST) sn = sin_fast(arg); else sn = sinf(arg);
        a[rt][0][r] = sn;
        continue;
      }
      if constexpr (FAST) sincos_fast(arg, sn, cs); else sincosf(arg, &sn, &cs);
      const float wc = OMEGA * cs;
      if constexpr (LAP) {
        float t2 = 0.f;
#pragma unroll
        for (int i = 0; i < NTAN; ++i) t2 = fmaf(a[rt][1 + i][r], a[rt][1 + i][r], t2);
        a[rt][S - 1][r] = wc * a[rt][S - 1][r] - OMEGA2 * sn * t2;
      }
#pragma unroll
      for (int i = 0; i < NTAN; ++i) a[rt][1 + i][r] *= wc;
      a[rt][0][r] = sn;
    }
  }
}

template <int NT, int S, bool LAP>
__device__ __forceinline__ void sine_jet(floatx4 (&a)[NT][S]) {
  float amax = 0.f;
#pragma unroll
  for (int rt = 0; rt < NT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) amax = fmaxf(amax, fabsf(OMEGA * a[rt][0][r]));
  if (wave_any_big(amax))
    sine_jet_impl<NT, S, LAP, false>(a);
  else
    sine_jet_impl<NT, S, LAP, true>(a);
}

template <int NT, int S>
__device__ __forceinline__ void save_streams(float* base, const floatx4 (&a)[NT][S], int lane) {
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int rt = 0; rt < NT; ++rt)
      *reinterpret_cast<floatx4*>(base + ((s * NT + rt) * 64 + lane) * 4) = a[rt][s];
}

template <int NT, int S, bool LAP>
__global__ __launch_bounds__(kThreads, 1) void jet_fwd_kernel(
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
// Sine reverse for one row-tile.  hb: adjoints of h-streams in, zb out (in place).
template <int S, bool LAP>
__device__ __forceinline__ void sine_rev(floatx4 (&hb)[S], const floatx4 (&zs)[S], const floatx4& sn,
                                         const floatx4& cs) {
  constexpr int NTAN = LAP ? S - 2 : S - 1;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float wc = OMEGA * cs[r], ws = OMEGA2 * sn[r];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < NTAN; ++i) dot = fmaf(zs[1 + i][r], hb[1 + i][r], dot);
    float zb = wc * hb[0][r] - ws * dot;
    if constexpr (LAP) {
      const float qh = hb[S - 1][r];
      float t2 = 0.f;
#pragma unroll
      for (int i = 0; i < NTAN; ++i) t2 = fmaf(zs[1 + i][r], zs[1 + i][r], t2);
      zb -= qh * (ws * zs[S - 1][r] + OMEGA3 * cs[r] * t2);
#pragma unroll
      for (int i = 0; i < NTAN; ++i) hb[1 + i][r] = wc * hb[1 + i][r] - 2.f * ws * zs[1 + i][r] * qh;
      hb[S - 1][r] = wc * qh;
    } else {
#pragma unroll
      for (int i = 0; i < NTAN; ++i) hb[1 + i][r] *= wc;
    }
    hb[0][r] = zb;
  }
}

template <int NT>
__device__ __forceinline__ void load_z_sincos(const float* base, int S, int lane, floatx4 (&sn)[NT],
                                              floatx4 (&cs)[NT]) {
  floatx4 z[NT];
  float amax = 0.f;
#pragma unroll
  for (int rt = 0; rt < NT; ++rt) {
    z[rt] = *reinterpret_cast<const floatx4*>(base + (rt * 64 + lane) * 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) amax = fmaxf(amax, fabsf(OMEGA * z[rt][r]));
  }
  const bool big = wave_any_big(amax);
#pragma unroll
  for (int rt = 0; rt < NT; ++rt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a, b;
      if (big)
        sincosf(OMEGA * z[rt][r], &a, &b);
      else
        sincos_fast(OMEGA * z[rt][r], a, b);
      sn[rt][r] = a;
      cs[rt][r] = b;
    }
  }
}

// h-stream s of a sine layer (for the weight gradient of the layer above),
// rebuilt from saved z-streams + cached sin/cos.
template <int NT, int S, bool LAP>
__device__ __forceinline__ floatx4 h_stream(const float* base, int s, int rt, int lane, const floatx4& sn,
                                            const floatx4& cs) {
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  if (s == 0) return sn;
  const floatx4 zs = *reinterpret_cast<const floatx4*>(base + ((s * NT + rt) * 64 + lane) * 4);
  floatx4 out;
  if (LAP && s == S - 1) {
    floatx4 t2 = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < NTAN; ++i) {
      const floatx4 t = *reinterpret_cast<const floatx4*>(base + (((1 + i) * NT + rt) * 64 + lane) * 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) t2[r] = fmaf(t[r], t[r], t2[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) out[r] = OMEGA * cs[r] * zs[r] - OMEGA2 * sn[r] * t2[r];
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) out[r] = OMEGA * cs[r] * zs[r];
  }
  return out;
}

template <int NT, int S, bool LAP>
__global__ __launch_bounds__(kThreads, 1) void jet_bwd_kernel(
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

// ---------------------------------------------------------------------------
// partial reduction + Adam
// ---------------------------------------------------------------------------
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
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    if (advance_step) st[INSR_OPT_STEP] = st[INSR_OPT_STEP] + 1.f;
    if (!loss) return;  // advance-only (optimiser without a scheduler)
    const float cur = *loss;
    float best = st[INSR_OPT_BEST];
    float bad = st[INSR_OPT_BAD];
    // torch: a < best * (1 - threshold), threshold = 1e-4 (python double math)
    if ((double)cur < (double)best * (1.0 - 1e-4)) {
      best = cur;
      bad = 0.f;
    } else {
      bad += 1.f;
    }
    if (bad > (float)patience) {
      const double old = st[INSR_OPT_LR];
      double nw = old * (double)st[INSR_OPT_FACTOR];
      if (nw < (double)st[INSR_OPT_MINLR]) nw = st[INSR_OPT_MINLR];
      if (old - nw > 1e-8) st[INSR_OPT_LR] = (float)nw;
      bad = 0.f;
    }
    st[INSR_OPT_BEST] = best;
    st[INSR_OPT_BAD] = bad;
  }
}

struct AdamList {
  float* p[INSR_ADAM_MAX_TENSORS];
  const float* g[INSR_ADAM_MAX_TENSORS];
  float* m[INSR_ADAM_MAX_TENSORS];
  float* v[INSR_ADAM_MAX_TENSORS];
  long n[INSR_ADAM_MAX_TENSORS];
  long start[INSR_ADAM_MAX_TENSORS + 1];  // prefix sums of n
  int count;
};

// One launch over up to INSR_ADAM_MAX_TENSORS flat buffers.  The step t used is
// st[STEP] + step_offset (the plateau kernel advances st[STEP] after the update,
// so the bias corrections need no separate prepare launch); torch's op order:
//   m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
//   p.addcdiv_(m, sqrt(v)/sqrt(1-b2^t) + eps, -lr/(1-b1^t))
__global__ void adam_multi_kernel(AdamList L, const float* __restrict__ st, float b1, float b2, float eps,
                                  int step_offset) {
  __shared__ float sc[2];
  if (threadIdx.x == 0) {
    const double t = (double)st[INSR_OPT_STEP] + (double)step_offset;
    sc[0] = (float)((double)st[INSR_OPT_LR] / (1.0 - pow((double)b1, t)));
    sc[1] = (float)sqrt(1.0 - pow((double)b2, t));
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
    const float g = L.g[k][i];
    const float m0 = L.m[k][i];
    const float mi = m0 + w1 * (g - m0);
    const float vi = L.v[k][i] * b2 + w2 * g * g;
    L.m[k][i] = mi;
    L.v[k][i] = vi;
    const float denom = sqrtf(vi) / bc2s + eps;
    L.p[k][i] = L.p[k][i] - step_size * (mi / denom);
  }
}

// ---------------------------------------------------------------------------
// host dispatch
// ---------------------------------------------------------------------------
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
  return -1;
}

size_t fwd_lds(int NT) { return (size_t)(16 * NT) * (16 * NT + 8) * sizeof(float); }
size_t bwd_lds(int NT) {
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
    (void)hipFuncSetAttribute((const void*)jet_fwd_kernel<NT, S, LAP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((jet_fwd_kernel<NT, S, LAP>), dim3(nb), dim3(kThreads), lds, st, x, N, din, dout, L, prm, y,
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
    (void)hipFuncSetAttribute((const void*)jet_bwd_kernel<NT, S, LAP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((jet_bwd_kernel<NT, S, LAP>), dim3(nb), dim3(kThreads), lds, st, x, N, din, dout, L, prm,
                     act, gy, gdy, glap, part, P);
  return (int)hipGetLastError();
}

// (S, LAP) combinations: value (1), grad d=1..3 (2..4), lap d=1,2 (3,4)
#define INSR_DISPATCH(NTV, FN, ...)                                  \
  switch (S * 2 + (LAP ? 1 : 0)) {                                   \
    case 2: return FN<NTV, 1, false>(__VA_ARGS__);                   \
    case 4: return FN<NTV, 2, false>(__VA_ARGS__);                   \
    case 6: return FN<NTV, 3, false>(__VA_ARGS__);                   \
    case 8: return FN<NTV, 4, false>(__VA_ARGS__);                   \
    case 7: return FN<NTV, 3, true>(__VA_ARGS__);                    \
    case 9: return FN<NTV, 4, true>(__VA_ARGS__);                    \
    default: return INSR_EINVAL;                                     \
  }

int dispatch_fwd(int NT, int S, bool LAP, const float* x, int N, int din, int dout, int L, const float* prm,
                 float* y, float* dy, float* lap, float* act, hipStream_t st) {
  switch (NT) {
    case 2: INSR_DISPATCH(2, launch_fwd, x, N, din, dout, L, prm, y, dy, lap, act, st)
    case 4: INSR_DISPATCH(4, launch_fwd, x, N, din, dout, L, prm, y, dy, lap, act, st)
    case 8: INSR_DISPATCH(8, launch_fwd, x, N, din, dout, L, prm, y, dy, lap, act, st)
    default: return INSR_EWIDTH;
  }
}

int dispatch_bwd(int NT, int S, bool LAP, const float* x, int N, int din, int dout, int L, const float* prm,
                 const float* act, const float* gy, const float* gdy, const float* glap, float* part, long P,
                 hipStream_t st) {
  switch (NT) {
    case 2: INSR_DISPATCH(2, launch_bwd, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    case 4: INSR_DISPATCH(4, launch_bwd, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    case 8: INSR_DISPATCH(8, launch_bwd, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    default: return INSR_EWIDTH;
  }
}

bool shape_ok(int din, int dout, int L, int width, int mode) {
  if (din < 1 || din > 3 || dout < 1 || dout > 3 || L < 0 || L > 64) return false;
  if (nt_for(width) < 0) return false;
  const int S = streams_for(din, mode);
  if (S < 1 || S > 4) return false;
  if (mode == INSR_MODE_LAP && din > 2) return false;
  return true;
}

}  // namespace

extern "C" {

int insr_version(void) { return 100; }

long insr_siren_param_count(int din, int dout, int L, int W) {
  return (long)W * din + W + (long)L * ((long)W * W + W) + (long)dout * W + dout;
}

int insr_siren_supported(int din, int dout, int L, int W, int mode) { return shape_ok(din, dout, L, W, mode) ? 1 : 0; }

long insr_jet_act_bytes(long n, int din, int L, int W, int mode) {
  const int S = streams_for(din, mode);
  if (S < 0 || n < 0) return INSR_EINVAL;
  const long tiles = ((n + kPts - 1) / kPts) * kWaves;
  return (long)(L + 1) * tiles * 16 * W * S * (long)sizeof(float);
}

long insr_jet_partial_bytes(long n, int din, int dout, int L, int W) {
  const long nb = (n + kPts - 1) / kPts;
  return nb * insr_siren_param_count(din, dout, L, W) * (long)sizeof(float);
}

int insr_siren_jet_fwd(const float* x, long n, int din, int dout, int L, int W, int mode, const float* params,
                       float* y, float* dy, float* lap, float* act, void* stream) {
  if (!shape_ok(din, dout, L, W, mode) || n < 0 || n > 0x7fffffffL) return INSR_EINVAL;
  if (n == 0) return 0;
  if (!x || !params || !y) return INSR_EINVAL;
  if (mode != INSR_MODE_VALUE && !dy) return INSR_EINVAL;
  if (mode == INSR_MODE_LAP && !lap) return INSR_EINVAL;
  const int S = streams_for(din, mode);
  return dispatch_fwd(nt_for(W), S, mode == INSR_MODE_LAP, x, (int)n, din, dout, L, params, y, dy, lap, act,
                      (hipStream_t)stream);
}

int insr_siren_jet_bwd(const float* x, long n, int din, int dout, int L, int W, int mode, const float* params,
                       const float* act, const float* gy, const float* gdy, const float* glap, float* partial,
                       void* stream) {
  if (!shape_ok(din, dout, L, W, mode) || n < 0 || n > 0x7fffffffL) return INSR_EINVAL;
  if (n == 0) return 0;
  if (!x || !params || !act || !partial) return INSR_EINVAL;
  const long P = insr_siren_param_count(din, dout, L, W);
  const int S = streams_for(din, mode);
  return dispatch_bwd(nt_for(W), S, mode == INSR_MODE_LAP, x, (int)n, din, dout, L, params, act, gy, gdy, glap,
                      partial, P, (hipStream_t)stream);
}

int insr_jet_partial_blocks(long n) { return n <= 0 ? 0 : (int)((n + kPts - 1) / kPts); }

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

int insr_adam_step_multi(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                         float* const* exp_avg_sq, const long* sizes, const float* st, float b1, float b2,
                         float eps, int step_offset, void* stream) {
  if (count < 1 || count > INSR_ADAM_MAX_TENSORS || !st) return INSR_EINVAL;
  AdamList L;
  L.count = count;
  L.start[0] = 0;
  for (int k = 0; k < count; ++k) {
    if (!params[k] || !grads[k] || !exp_avg[k] || !exp_avg_sq[k] || sizes[k] < 0) return INSR_EINVAL;
    L.p[k] = params[k];
    L.g[k] = grads[k];
    L.m[k] = exp_avg[k];
    L.v[k] = exp_avg_sq[k];
    L.n[k] = sizes[k];
    L.start[k + 1] = L.start[k] + sizes[k];
  }
  const long total = L.start[count];
  if (total == 0) return 0;
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
