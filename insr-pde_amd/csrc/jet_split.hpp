// jet_split.hpp -- "tile-split" SIREN jet kernels (instantiated by jet_split_fwd.hip
// and jet_split_bwd.hip, one translation unit per direction).
//
// A block owns T 16-point tiles and splits the OUTPUT NEURONS of every layer over
// its waves: wave w owns row tiles w*RPW .. w*RPW+RPW-1 (16 neurons each), with
// WV = min(NT, 8) waves per block and RPW = NT / WV.  Each wave's serial chain
// per layer is therefore 1/WV of a layer, the per-wave register state is small
// (2-3 waves per SIMD), and the T tiles of a block share every W fetch, every
// barrier and ONE partial-gradient row.
//
//  forward   activations of the T tiles live in LDS point-major [t][s][p][W+8]
//            (conflict-free ds_read_b128 as the MFMA B operand); each wave holds
//            its W rows (the A operand) in registers for the layer.  Per layer:
//            read + MFMA / barrier / save z, sine jet, write h / barrier.
//  backward  per layer: sine reverse in registers -> zb and h_{j-1} of all T tiles
//            into point-major LDS planes -> this wave's dW rows (K = 16T points x
//            S streams, MFMA) -> propagation W^T zb for this wave's rows.
//
// Saved activations use the wave-tile layout (jet_common.hpp) with the same tile
// count (ceil(N/64)*4, and T divides 4), so the forward and backward variants are
// interchangeable.
#pragma once
#include "jet_common.hpp"

namespace insr {

template <int NT>
struct SplitGeo {
  static constexpr int W = 16 * NT;
  static constexpr int WV = NT < 8 ? NT : 8;  // waves per block
  static constexpr int RPW = NT / WV;         // row tiles per wave
  static constexpr int LDH = W + 8;           // point-major LDS row (floats)
  static constexpr int THREADS = 64 * WV;
  static constexpr int PLANE = 16 * LDH;      // one (tile, stream) plane
};

constexpr size_t kLdsMax = 163840;  // 160 KB per CU on gfx950

template <int NT, int S, int T>
constexpr size_t fwd_split_lds_bytes() {
  return (size_t)T * S * SplitGeo<NT>::PLANE * sizeof(float);
}
// backward: zb planes point-major with row W+8 (conflict-free ds_read_b128 rows for
// the propagation B operand, 4 b32 column reads for the dW A operand); h planes
// NEURON-major [m][16 points] so the dW B operand (4 consecutive points of one
// neuron) is one ds_read_b128.  The 16-B slot of (m, p) is XOR-swizzled by
// ((m>>1) ^ (m>>2)) & 3: conflict-free b128 reads, 2-way b32 writes, no padding.
__device__ __forceinline__ int hT_index(int m, int p) { return m * 16 + ((((p >> 2) ^ (m >> 1) ^ (m >> 2)) & 3) << 2) + (p & 3); }
template <int NT, int S, int T>
constexpr size_t bwd_split_lds_bytes() {
  return (size_t)T * S * (SplitGeo<NT>::PLANE + 16 * 16 * NT) * sizeof(float);
}

template <int NT, int S, bool LAP, int T>
__global__ __launch_bounds__(SplitGeo<NT>::THREADS) void jet_fwd_split(
    const float* __restrict__ x, int N, int din, int dout, int L, const float* __restrict__ prm,
    float* __restrict__ y, float* __restrict__ dy, float* __restrict__ lap, float* __restrict__ act) {
  using G = SplitGeo<NT>;
  constexpr int W = G::W, RPW = G::RPW, LDH = G::LDH, WV = G::WV, PLANE = G::PLANE;
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int ntiles = ((N + 63) / 64) * 4;
  const int tile0 = blockIdx.x * T;
  const int rt0 = wave * RPW;

  float xv[T][3];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int p = (tile0 + t) * 16 + c;
    for (int k = 0; k < 3; ++k) xv[t][k] = (p < N && k < din) ? x[(long)p * din + k] : 0.f;
  }

  floatx4 a[T][RPW][S];
  {  // layer 0 (K = d_in: VALU)
    const float* W0 = prm;
    const float* b0 = prm + (long)W * din;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * (rt0 + i) + 4 * g + r;
        const float bn = b0[n];
        float w0[3] = {0.f, 0.f, 0.f};
        for (int k = 0; k < din; ++k) w0[k] = W0[n * din + k];
#pragma unroll
        for (int t = 0; t < T; ++t) {
          float z = bn;
          for (int k = 0; k < din; ++k) z = fmaf(w0[k], xv[t][k], z);
          a[t][i][0][r] = z;
#pragma unroll
          for (int k = 0; k < NTAN; ++k) a[t][i][1 + k][r] = w0[k];
          if constexpr (LAP) a[t][i][S - 1][r] = 0.f;
        }
      }
    }
  }
  for (int j = 0; j <= L; ++j) {
    if (j > 0) {
      // hidden layer j: B operands (layer j-1 activations) from LDS, A = W rows in registers
      const float* Wj = prm + hidden_off(din, W, j);
      const float* bj = Wj + (long)W * W;
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        const int rt = rt0 + i;
        floatx4 wr[NT];
#pragma unroll
        for (int kt = 0; kt < NT; ++kt)
          wr[kt] = *reinterpret_cast<const floatx4*>(Wj + ((16 * rt + c) * W + 16 * kt + 4 * g));
        const floatx4 bias = *reinterpret_cast<const floatx4*>(bj + 16 * rt + 4 * g);
#pragma unroll
        for (int t = 0; t < T; ++t) {
          a[t][i][0] = bias;
#pragma unroll
          for (int s = 1; s < S; ++s) a[t][i][s] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        // consecutive MFMAs go to independent accumulators (the f32 16x16x4 MFMA has a
        // 40-cycle dependent latency vs a 32-cycle issue); each accumulator's k-order is
        // unchanged, so results are bit-identical to the plain loop
#pragma unroll
        for (int kt = 0; kt < NT; ++kt) {
          if constexpr (S >= 2) {
#pragma unroll
            for (int t = 0; t < T; ++t) {
              floatx4 hv[S];
#pragma unroll
              for (int s = 0; s < S; ++s)
                hv[s] = *reinterpret_cast<const floatx4*>(lds + (t * S + s) * PLANE + c * LDH + 16 * kt + 4 * g);
#pragma unroll
              for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int s = 0; s < S; ++s) a[t][i][s] = mfma4(wr[kt][r], hv[s][r], a[t][i][s]);
            }
          } else {
            floatx4 hv[T];
#pragma unroll
            for (int t = 0; t < T; ++t)
              hv[t] = *reinterpret_cast<const floatx4*>(lds + t * PLANE + c * LDH + 16 * kt + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int t = 0; t < T; ++t) a[t][i][0] = mfma4(wr[kt][r], hv[t][r], a[t][i][0]);
          }
        }
      }
      __syncthreads();  // every wave has read layer j-1
    }
    if (act) {  // the first layer: its value stream only (l0_rebuilt, jet_common.hpp)
      const int ns = l0_rebuilt(j, L) ? 1 : S;
#pragma unroll
      for (int t = 0; t < T; ++t) {
        float* base = act_base(act, j, ntiles, tile0 + t, S, NT);
#pragma unroll
        for (int i = 0; i < RPW; ++i)
#pragma unroll
          for (int s = 0; s < S; ++s)
            if (s < ns) *reinterpret_cast<floatx4*>(base + ((s * NT + rt0 + i) * 64 + lane) * 4) = a[t][i][s];
      }
    }
#pragma unroll
    for (int t = 0; t < T; ++t) sine_jet<RPW, S, LAP>(a[t]);
    if (j < L) {
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int i = 0; i < RPW; ++i)
#pragma unroll
          for (int s = 0; s < S; ++s)
            *reinterpret_cast<floatx4*>(lds + (t * S + s) * PLANE + c * LDH + 16 * (rt0 + i) + 4 * g) = a[t][i][s];
      __syncthreads();
    }
  }
  // output layer: each wave sums its own neurons; the waves combine through LDS
  // (the activation planes are dead: every wave passed the last read barrier)
  float* red = lds;  // [WV][T][S][3][16]
  const float* Wo = prm + out_off(din, W, L);
  const float* bo = Wo + (long)dout * W;
  for (int o = 0; o < dout; ++o) {
    float sv[T][S];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int s = 0; s < S; ++s) sv[t][s] = 0.f;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const floatx4 w4 = *reinterpret_cast<const floatx4*>(Wo + (o * W + 16 * (rt0 + i) + 4 * g));
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int s = 0; s < S; ++s) sv[t][s] = fmaf(w4[r], a[t][i][s][r], sv[t][s]);
    }
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int s = 0; s < S; ++s) {
        float v = sv[t][s];
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        if (g == 0) red[(((wave * T + t) * S + s) * 3 + o) * 16 + c] = v;
      }
  }
  __syncthreads();
  if (wave == 0 && g < T) {  // lane group g finishes tile g
    const int t = g;
    const int p = (tile0 + t) * 16 + c;
    if (p < N) {
      for (int o = 0; o < dout; ++o) {
        float tot[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
          tot[s] = 0.f;
#pragma unroll
          for (int w = 0; w < WV; ++w) tot[s] += red[(((w * T + t) * S + s) * 3 + o) * 16 + c];
        }
        y[(long)p * dout + o] = tot[0] + bo[o];
        if (dy)
          for (int k = 0; k < NTAN; ++k) dy[((long)p * dout + o) * din + k] = tot[1 + k];
        if constexpr (LAP) {
          if (lap) lap[(long)p * dout + o] = tot[S - 1];
        }
      }
    }
  }
}

template <int NT, int S, bool LAP, int T>
__global__ __launch_bounds__(SplitGeo<NT>::THREADS) void jet_bwd_split(
    const float* __restrict__ x, int N, int din, int dout, int L, const float* __restrict__ prm,
    const float* __restrict__ act, const float* __restrict__ gy, const float* __restrict__ gdy,
    const float* __restrict__ glap, float* __restrict__ part, long P) {
  using G = SplitGeo<NT>;
  constexpr int W = G::W, RPW = G::RPW, LDH = G::LDH, PLANE = G::PLANE;
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  // both planes point-major [t][s][16 points][LDH]: zbp is read as b128 rows (the
  // propagation B operand) and as 4 b32 columns (the dW A operand); hpp as columns
  constexpr int PLANEH = 16 * W;
  float* zbp = lds;                  // zb of layer j      [t][s][p][LDH]
  float* hpp = lds + T * S * PLANE;  // h of layer j-1     [t][s][m][16] (hT_index)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int ntiles = ((N + 63) / 64) * 4;
  const int tile0 = blockIdx.x * T;
  // saved streams of slot t: a slot past the batch's last tile re-reads tile0 (the forward, whose
  // T may be smaller, never wrote it; its adjoints are zero, so it contributes nothing)
  const int tiles_n = (N + 15) / 16;
  auto tl = [&](int t) { return tile0 + t < tiles_n ? tile0 + t : tile0; };
  const int rt0 = wave * RPW;
  float* mypart = part + (long)blockIdx.x * P;

  float xv[T][3];
  float ga[T][S][3];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int p = (tile0 + t) * 16 + c;
    const bool valid = p < N;
    for (int k = 0; k < 3; ++k) xv[t][k] = (valid && k < din) ? x[(long)p * din + k] : 0.f;
#pragma unroll
    for (int s = 0; s < S; ++s)
      for (int o = 0; o < 3; ++o) ga[t][s][o] = 0.f;
    if (valid) {
      for (int o = 0; o < dout; ++o) {
        if (gy) ga[t][0][o] = gy[(long)p * dout + o];
        if (gdy)
          for (int k = 0; k < NTAN; ++k) ga[t][1 + k][o] = gdy[((long)p * dout + o) * din + k];
        if constexpr (LAP) {
          if (glap) ga[t][S - 1][o] = glap[(long)p * dout + o];
        }
      }
    }
  }

  // sin/cos of omega * z_layer for this wave's rows of all T tiles (one uniform
  // fast/libm decision for the wave)
  auto load_sc = [&](int layer, floatx4(&s_)[T][RPW], floatx4(&c_)[T][RPW]) {
    floatx4 z[T][RPW];
    float amax = 0.f;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const float* base = act_base(act, layer, ntiles, tl(t), S, NT);
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        z[t][i] = *reinterpret_cast<const floatx4*>(base + ((rt0 + i) * 64 + lane) * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) amax = fmaxf(amax, fabsf(OMEGA * z[t][i][r]));
      }
    }
    const bool big = wave_any_big(amax);
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int i = 0; i < RPW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float sv, cv;
          if (big)
            sincosf(OMEGA * z[t][i][r], &sv, &cv);
          else
            sincos_fast(OMEGA * z[t][i][r], sv, cv);
          s_[t][i][r] = sv;
          c_[t][i][r] = cv;
        }
  };

  // ---- output layer ----
  floatx4 sn[T][RPW], cs[T][RPW];
  load_sc(L, sn, cs);
  const float* Wo = prm + out_off(din, W, L);
  const long wo_off = out_off(din, W, L);
  floatx4 hb[T][RPW][S];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int s = 0; s < S; ++s) hb[t][i][s] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int o = 0; o < dout; ++o) {
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int rt = rt0 + i;
      const floatx4 w4 = *reinterpret_cast<const floatx4*>(Wo + (o * W + 16 * rt + 4 * g));
      floatx4 acc4 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const float* baseL = act_base(act, L, ntiles, tl(t), S, NT);
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const floatx4 hs = h_stream<NT, S, LAP>(baseL, s, rt, lane, sn[t][i], cs[t][i]);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            acc4[r] = fmaf(ga[t][s][o], hs[r], acc4[r]);
            hb[t][i][s][r] = fmaf(w4[r], ga[t][s][o], hb[t][i][s][r]);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = sum16(acc4[r]);
        if (c == 0) mypart[wo_off + (long)o * W + 16 * rt + 4 * g + r] = v;
      }
    }
    if (wave == 0) {  // db_out[o]: every point counted once (lane group g == 0)
      float v = 0.f;
#pragma unroll
      for (int t = 0; t < T; ++t) v += (g == 0) ? ga[t][0][o] : 0.f;
      v = sum16(v);
      if (lane == 0) mypart[wo_off + (long)dout * W + o] = v;
    }
  }

  // ---- sine layers j = L .. 0 ----
  // Small register states hoist the propagation's W^T operand loads to the top of
  // the layer, so their latency overlaps the sine reverse, the LDS exchange and dW.
  constexpr bool kHoistWT = RPW == 1 && T * S <= 4;
  float wt[kHoistWT ? NT : 1][4];
  // z-streams s >= 1 of the layer the next sine reverse needs: loaded once (with the h
  // planes of the layer above) and kept in registers when the state is small enough
  constexpr bool kKeepZ = S > 1 && T * (S - 1) * RPW <= 3;
  floatx4 zk[kKeepZ ? T : 1][kKeepZ ? RPW : 1][kKeepZ ? S : 1];
  if constexpr (kKeepZ) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const float* baseL = act_base(act, L, ntiles, tl(t), S, NT);
#pragma unroll
      for (int i = 0; i < RPW; ++i)
#pragma unroll
        for (int s = 1; s < S; ++s)
          zk[t][i][s] = load_zs<NT, S, LAP>(baseL, s, rt0 + i, lane, l0_rebuilt(L, L), prm, din);
    }
  }
  for (int j = L; j >= 0; --j) {
    INSR_STAMP(L - j, 0);
    if constexpr (kHoistWT) {
      if (j > 0) {
        const float* Wj = prm + hidden_off(din, W, j);
#pragma unroll
        for (int kt = 0; kt < NT; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) wt[kt][r] = Wj[(16 * kt + 4 * g + r) * W + 16 * rt0 + c];
      }
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const float* basej = act_base(act, j, ntiles, tl(t), S, NT);
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        floatx4 zs[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
          if constexpr (kKeepZ)
            zs[s] = (s == 0) ? floatx4{0.f, 0.f, 0.f, 0.f} : zk[t][i][s];
          else
            zs[s] = (s == 0) ? floatx4{0.f, 0.f, 0.f, 0.f}
                             : load_zs<NT, S, LAP>(basej, s, rt0 + i, lane, l0_rebuilt(j, L), prm, din);
        }
        sine_rev<S, LAP>(hb[t][i], zs, sn[t][i], cs[t][i]);
      }
    }
    const long boff = (j == 0) ? (long)W * din : hidden_off(din, W, j) + (long)W * W;
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = 0.f;
#pragma unroll
        for (int t = 0; t < T; ++t) v += hb[t][i][0][r];
        v = sum16(v);
        if (c == 0) mypart[boff + 16 * (rt0 + i) + 4 * g + r] = v;
      }
    INSR_STAMP(L - j, 1);
    if (j == 0) {
#pragma unroll
      for (int i = 0; i < RPW; ++i)
        for (int k = 0; k < din; ++k)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = 0.f;
#pragma unroll
            for (int t = 0; t < T; ++t) {
              v = fmaf(hb[t][i][0][r], xv[t][k], v);
              if (k < NTAN) v += hb[t][i][1 + k][r];
            }
            v = sum16(v);
            if (c == 0) mypart[(long)(16 * (rt0 + i) + 4 * g + r) * din + k] = v;
          }
      break;
    }
    // sin/cos of z_{j-1}: h_{j-1} now, and the sine reverse of the next iteration
    floatx4 snp[T][RPW], csp[T][RPW];
    load_sc(j - 1, snp, csp);
    INSR_STAMP(L - j, 2);
    __syncthreads();  // the previous layer's LDS readers are done
    INSR_STAMP(L - j, 3);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const float* basep = act_base(act, j - 1, ntiles, tl(t), S, NT);
#pragma unroll
      for (int i = 0; i < RPW; ++i)
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int col = 16 * (rt0 + i) + 4 * g;
          *reinterpret_cast<floatx4*>(zbp + (t * S + s) * PLANE + c * LDH + col) = hb[t][i][s];
          floatx4 hs;
          if constexpr (kKeepZ) {
            hs = h_from_z<NT, S, LAP>(basep, s, rt0 + i, lane, snp[t][i], csp[t][i], zk[t][i], l0_rebuilt(j - 1, L),
                                      prm, din);
          } else {
            hs = h_stream<NT, S, LAP>(basep, s, rt0 + i, lane, snp[t][i], csp[t][i], l0_rebuilt(j - 1, L), prm, din);
          }
          float* hp_ts = hpp + (t * S + s) * PLANEH;
#pragma unroll
          for (int r = 0; r < 4; ++r) hp_ts[hT_index(col + r, c)] = hs[r];
        }
    }
    INSR_STAMP(L - j, 4);
    __syncthreads();
    INSR_STAMP(L - j, 5);
    {  // dW_j, this wave's rows: K = 16T points x S streams (k = point 4g + r)
      float* dW = mypart + hidden_off(din, W, j);
      constexpr int CTC = NT < 4 ? NT : 4;  // column tiles per accumulator pass (register budget)
#pragma unroll 1
      for (int i = 0; i < RPW; ++i) {
        const int rt = rt0 + i;
#pragma unroll 1
        for (int ct0 = 0; ct0 < NT; ct0 += CTC) {
          floatx4 dacc[CTC];
#pragma unroll
          for (int ct = 0; ct < CTC; ++ct) dacc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int t = 0; t < T; ++t)
#pragma unroll
            for (int s = 0; s < S; ++s) {
              const float* zb_ts = zbp + (t * S + s) * PLANE;
              const float* hp_ts = hpp + (t * S + s) * PLANEH;
              floatx4 a4, hv[CTC];
#pragma unroll
              for (int r = 0; r < 4; ++r) a4[r] = zb_ts[(4 * g + r) * LDH + 16 * rt + c];
#pragma unroll
              for (int ct = 0; ct < CTC; ++ct)  // h(points 4g..4g+3, neuron 16ct + c)
                hv[ct] = *reinterpret_cast<const floatx4*>(hp_ts + hT_index(16 * (ct0 + ct) + c, 4 * g));
              // r outer: CTC independent accumulators between dependent MFMAs
#pragma unroll
              for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int ct = 0; ct < CTC; ++ct) dacc[ct] = mfma4(a4[r], hv[ct][r], dacc[ct]);
            }
#pragma unroll
          for (int ct = 0; ct < CTC; ++ct)
#pragma unroll
            for (int r = 0; r < 4; ++r) dW[(16 * rt + 4 * g + r) * W + 16 * (ct0 + ct) + c] = dacc[ct][r];
        }
      }
    }
    INSR_STAMP(L - j, 6);
    {  // propagate: hb_{j-1}[m] (this wave's rows) = sum_n W_j[n][m] zb[n]; A = W^T from L2
      const float* Wj = prm + hidden_off(din, W, j);
      floatx4 nh[T][RPW][S];
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int i = 0; i < RPW; ++i)
#pragma unroll
          for (int s = 0; s < S; ++s) nh[t][i][s] = floatx4{0.f, 0.f, 0.f, 0.f};
      constexpr int KU = NT > 8 ? 2 : NT;  // bounded unroll: W^T loads in flight
#pragma unroll KU
      for (int kt = 0; kt < NT; ++kt) {
        floatx4 wa[RPW];
#pragma unroll
        for (int i = 0; i < RPW; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if constexpr (kHoistWT)
              wa[i][r] = wt[kt][r];
            else
              wa[i][r] = Wj[(16 * kt + 4 * g + r) * W + 16 * (rt0 + i) + c];
          }
        if constexpr (S >= 2) {  // r outer over S (x RPW) independent accumulators
#pragma unroll
          for (int t = 0; t < T; ++t) {
            floatx4 b4[S];
#pragma unroll
            for (int s = 0; s < S; ++s)
              b4[s] = *reinterpret_cast<const floatx4*>(zbp + (t * S + s) * PLANE + c * LDH + 16 * kt + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int s = 0; s < S; ++s)
#pragma unroll
                for (int i = 0; i < RPW; ++i) nh[t][i][s] = mfma4(wa[i][r], b4[s][r], nh[t][i][s]);
          }
        } else {  // value jets: r outer over the T tiles
          floatx4 b4[T];
#pragma unroll
          for (int t = 0; t < T; ++t)
            b4[t] = *reinterpret_cast<const floatx4*>(zbp + t * PLANE + c * LDH + 16 * kt + 4 * g);
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < T; ++t)
#pragma unroll
              for (int i = 0; i < RPW; ++i) nh[t][i][0] = mfma4(wa[i][r], b4[t][r], nh[t][i][0]);
        }
      }
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
          sn[t][i] = snp[t][i];
          cs[t][i] = csp[t][i];
#pragma unroll
          for (int s = 0; s < S; ++s) hb[t][i][s] = nh[t][i][s];
        }
    }
    INSR_STAMP(L - j, 7);
  }
}

// ---------------------------------------------------------------------------
// launchers; T (tiles per block) is chosen on the host by split_tiles()
// ---------------------------------------------------------------------------
template <int NT, int S, bool LAP, int T>
int launch_fwd_split_t(const float* x, int N, int din, int dout, int L, const float* prm, float* y, float* dy,
                       float* lap, float* act, hipStream_t st) {
  constexpr size_t lds = fwd_split_lds_bytes<NT, S, T>();
  if constexpr (lds > kLdsMax) {
    return INSR_EINVAL;
  } else {
    const int nb = ((N + 15) / 16 + T - 1) / T;
    static const bool attr_set = ((void)hipFuncSetAttribute((const void*)jet_fwd_split<NT, S, LAP, T>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), true);  // once per instantiation (thread-safe static init)
    (void)attr_set;
    if (N < 0) {  // occupancy query (split_tiles): resident blocks per CU
      int occ = 0;
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)jet_fwd_split<NT, S, LAP, T>, SplitGeo<NT>::THREADS, lds);
      return occ;
    }
    hipLaunchKernelGGL((jet_fwd_split<NT, S, LAP, T>), dim3(nb), dim3(SplitGeo<NT>::THREADS), lds, st, x, N, din,
                       dout, L, prm, y, dy, lap, act);
    return (int)hipGetLastError();
  }
}

template <int NT, int S, bool LAP, int T>
int launch_bwd_split_t(const float* x, int N, int din, int dout, int L, const float* prm, const float* act,
                       const float* gy, const float* gdy, const float* glap, float* part, long P, hipStream_t st) {
  constexpr size_t lds = bwd_split_lds_bytes<NT, S, T>();
  if constexpr (lds > kLdsMax) {
    return INSR_EINVAL;
  } else {
    const int nb = ((N + 15) / 16 + T - 1) / T;
    static const bool attr_set = ((void)hipFuncSetAttribute((const void*)jet_bwd_split<NT, S, LAP, T>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), true);  // once per instantiation (thread-safe static init)
    (void)attr_set;
    if (N < 0) {  // occupancy query (split_tiles): resident blocks per CU
      int occ = 0;
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)jet_bwd_split<NT, S, LAP, T>, SplitGeo<NT>::THREADS, lds);
      return occ;
    }
    hipLaunchKernelGGL((jet_bwd_split<NT, S, LAP, T>), dim3(nb), dim3(SplitGeo<NT>::THREADS), lds, st, x, N, din,
                       dout, L, prm, act, gy, gdy, glap, part, P);
    return (int)hipGetLastError();
  }
}

}  // namespace insr
