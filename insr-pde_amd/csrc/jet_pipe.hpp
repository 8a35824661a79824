// jet_pipe.hpp -- software-pipelined tile-split backward (T >= 2 tiles per block).
//
// The tile-split backward (jet_split.hpp) runs every layer as
//   VALU phase  (sine reverse, sin/cos of z_{j-1}, h_{j-1} streams, LDS writes)
//   barrier
//   MFMA phase  (dW rows, W^T propagation)
// and since one block fills a CU, both waves of a SIMD sit in the same phase: the
// MFMA pipe idles through every VALU phase (s_memtime stamps: ~25% of a layer).
// Here the block's T tiles are split into two halves A and B that run half a layer
// apart, so every barrier interval holds the MFMA phase of one half AND the VALU
// phase of the other; the two waves of each SIMD take the two parts in opposite
// orders, so the MFMA chain of one overlaps the VALU work of the other:
//
//   V(A,L) | M(A,L) V(B,L) | M(B,L) V(A,L-1) | M(A,L-1) V(B,L-1) | ... | M(B,1) V(A,0) | V(B,0)
//
// Each half owns its LDS planes (written by V, read by the next M of that half), the
// dW accumulator carries from M(A,j) to M(B,j), the bias partial from V(A,j) to
// V(B,j).  Per-point arithmetic and every accumulation order over a half are those of
// jet_bwd_split; the sums over the two halves add in a fixed order (A then B).
#pragma once
#include <type_traits>

#include "jet_split.hpp"

namespace insr {

template <int NT, int S, bool LAP, int T>
__global__ __launch_bounds__(SplitGeo<NT>::THREADS) void jet_bwd_pipe(
    const float* __restrict__ x, int N, int din, int dout, int L, const float* __restrict__ prm,
    const float* __restrict__ act, const float* __restrict__ gy, const float* __restrict__ gdy,
    const float* __restrict__ glap, float* __restrict__ part, long P, int order) {
  static_assert(NT <= 8 && T % 2 == 0, "pipelined backward: one row tile per wave, an even tile count");
  using G = SplitGeo<NT>;
  constexpr int W = G::W, LDH = G::LDH, PLANE = G::PLANE, PLANEH = 16 * W;
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  constexpr int TH = T / 2;  // tiles per half
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* zbp = lds;                  // zb of the half's current layer   [t][s][p][LDH]
  float* hpp = lds + T * S * PLANE;  // h of the layer below            [t][s][m][16] (hT_index)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int ntiles = ((N + 63) / 64) * 4;
  const int tile0 = blockIdx.x * T;
  const int rt = wave;  // this wave's row tile
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
#pragma unroll
      for (int o = 0; o < 3; ++o) {  // constant trip count: ga stays in registers
        if (o >= dout) break;
        if (gy) ga[t][0][o] = gy[(long)p * dout + o];
        if (gdy)
          for (int k = 0; k < NTAN; ++k) ga[t][1 + k][o] = gdy[((long)p * dout + o) * din + k];
        if constexpr (LAP) {
          if (glap) ga[t][S - 1][o] = glap[(long)p * dout + o];
        }
      }
    }
  }

  // sin/cos of omega * z_layer, this wave's rows, tiles of half h: the fast path
  // unconditionally, libm only for a wave holding an argument beyond its range
  auto load_sc = [&](int layer, int h, floatx4(&s_)[TH], floatx4(&c_)[TH]) __attribute__((always_inline)) {
    floatx4 z[TH];
    float amax = 0.f;
#pragma unroll
    for (int tt = 0; tt < TH; ++tt) {
      const float* base = act_base(act, layer, ntiles, tile0 + h * TH + tt, S, NT);
      z[tt] = *reinterpret_cast<const floatx4*>(base + (rt * 64 + lane) * 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        amax = fmaxf(amax, fabsf(OMEGA * z[tt][r]));
        float sv, cv;
        sincos_fast(OMEGA * z[tt][r], sv, cv);
        s_[tt][r] = sv;
        c_[tt][r] = cv;
      }
    }
    if (wave_any_big(amax)) {
#pragma unroll
      for (int tt = 0; tt < TH; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float sv, cv;
          sincosf(OMEGA * z[tt][r], &sv, &cv);
          s_[tt][r] = sv;
          c_[tt][r] = cv;
        }
    }
  };

  // ---- output layer (all tiles) ----
  // sin/cos of the output-facing layer (recomputed per use below: with the pipelined
  // schedule VALU is off the critical path, registers are not)
  floatx4 sn[2][TH], cs[2][TH];
  load_sc(L, 0, sn[0], cs[0]);
  load_sc(L, 1, sn[1], cs[1]);
  const float* Wo = prm + out_off(din, W, L);
  const long wo_off = out_off(din, W, L);
  floatx4 hb[2][TH][S];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int tt = 0; tt < TH; ++tt)
#pragma unroll
      for (int s = 0; s < S; ++s) hb[h][tt][s] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    if (o >= dout) break;
    const floatx4 w4 = *reinterpret_cast<const floatx4*>(Wo + (long)o * W + 16 * rt + 4 * g);
    floatx4 acc4 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int h = t / TH, tt = t % TH;
      const float* baseL = act_base(act, L, ntiles, tile0 + t, S, NT);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const floatx4 hs = h_stream<NT, S, LAP>(baseL, s, rt, lane, sn[h][tt], cs[h][tt]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc4[r] = fmaf(ga[t][s][o], hs[r], acc4[r]);
          hb[h][tt][s][r] = fmaf(w4[r], ga[t][s][o], hb[h][tt][s][r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = sum16(acc4[r]);
      if (c == 0) mypart[wo_off + (long)o * W + 16 * rt + 4 * g + r] = v;
    }
    if (wave == 0) {  // db_out[o]: every point counted once (lane group g == 0)
      float v = 0.f;
#pragma unroll
      for (int t = 0; t < T; ++t) v += (g == 0) ? ga[t][0][o] : 0.f;
      v = sum16(v);
      if (lane == 0) mypart[wo_off + (long)dout * W + o] = v;
    }
  }

  float bsum[4];        // bias partial of half A, completed by half B
  float w0sum[3][4];    // first-layer weight partial of half A (j = 0)
  floatx4 dacc[NT];     // dW rows of this wave: half A's contribution, completed by half B

  // ---- V(h, j): sine reverse, bias, then (j >= 1) sin/cos(z_{j-1}) and the LDS planes
  // of half h, or (LAST: j == 0) the first layer's weight gradient ----
  auto V = [&](auto H, auto LASTC, int j) __attribute__((always_inline)) {
    constexpr int h = decltype(H)::value;
    constexpr bool LAST = decltype(LASTC)::value;
    floatx4 snj[TH], csj[TH];
    load_sc(j, h, snj, csj);
#pragma unroll
    for (int tt = 0; tt < TH; ++tt) {
      const float* basej = act_base(act, j, ntiles, tile0 + h * TH + tt, S, NT);
      floatx4 zs[S];
#pragma unroll
      for (int s = 0; s < S; ++s)
        zs[s] = (s == 0) ? floatx4{0.f, 0.f, 0.f, 0.f}
                         : *reinterpret_cast<const floatx4*>(basej + ((s * NT + rt) * 64 + lane) * 4);
      sine_rev<S, LAP>(hb[h][tt], zs, snj[tt], csj[tt]);
    }
    const long boff = LAST ? (long)W * din : hidden_off(din, W, j) + (long)W * W;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = 0.f;
#pragma unroll
      for (int tt = 0; tt < TH; ++tt) v += hb[h][tt][0][r];
      if constexpr (h == 0) {
        bsum[r] = v;
      } else {
        v = sum16(bsum[r] + v);
        if (c == 0) mypart[boff + 16 * rt + 4 * g + r] = v;
      }
    }
    if constexpr (LAST) {  // first layer: dW0 = sum_points zb0 x + tb (K = d_in, VALU)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        if (k >= din) break;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = 0.f;
#pragma unroll
          for (int tt = 0; tt < TH; ++tt) {
            v = fmaf(hb[h][tt][0][r], xv[h * TH + tt][k], v);
            if (k < NTAN) v += hb[h][tt][1 + k][r];
          }
          if constexpr (h == 0) {
            w0sum[k][r] = v;
          } else {
            v = sum16(w0sum[k][r] + v);
            if (c == 0) mypart[(long)(16 * rt + 4 * g + r) * din + k] = v;
          }
        }
      }
      return;
    }
    floatx4 snp[TH], csp[TH];
    load_sc(j - 1, h, snp, csp);
#pragma unroll
    for (int tt = 0; tt < TH; ++tt) {
      const int t = h * TH + tt;
      const float* basep = act_base(act, j - 1, ntiles, tile0 + t, S, NT);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int col = 16 * rt + 4 * g;
        *reinterpret_cast<floatx4*>(zbp + (t * S + s) * PLANE + c * LDH + col) = hb[h][tt][s];
        const floatx4 hs = h_stream<NT, S, LAP>(basep, s, rt, lane, snp[tt], csp[tt]);
        float* hp_ts = hpp + (t * S + s) * PLANEH;
#pragma unroll
        for (int r = 0; r < 4; ++r) hp_ts[hT_index(col + r, c)] = hs[r];
      }
    }
  };

  // ---- M(h, j): dW rows (half h's points) and the W^T propagation of half h ----
  auto M = [&](auto H, int j) __attribute__((always_inline)) {
    constexpr int h = decltype(H)::value;
    if constexpr (h == 0) {
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) dacc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int tt = 0; tt < TH; ++tt) {
      const int t = h * TH + tt;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const float* zb_ts = zbp + (t * S + s) * PLANE;
        const float* hp_ts = hpp + (t * S + s) * PLANEH;
        floatx4 a4;
#pragma unroll
        for (int r = 0; r < 4; ++r) a4[r] = zb_ts[(4 * g + r) * LDH + 16 * rt + c];
#pragma unroll
        for (int c0 = 0; c0 < NT; c0 += 4) {
          constexpr int CC = NT < 4 ? NT : 4;
          floatx4 hv[CC];
#pragma unroll
          for (int q = 0; q < CC; ++q) hv[q] = *reinterpret_cast<const floatx4*>(hp_ts + hT_index(16 * (c0 + q) + c, 4 * g));
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < CC; ++q) dacc[c0 + q] = mfma4(a4[r], hv[q][r], dacc[c0 + q]);
        }
      }
    }
    if constexpr (h == 1) {
      float* dW = mypart + hidden_off(din, W, j);
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) dW[(long)(16 * rt + 4 * g + r) * W + 16 * ct + c] = dacc[ct][r];
    }
    // propagation: hb_{j-1}[m] (this wave's rows) = sum_n W_j[n][m] zb[n]
    const float* Wj = prm + hidden_off(din, W, j);
    floatx4 nh[TH][S];
#pragma unroll
    for (int tt = 0; tt < TH; ++tt)
#pragma unroll
      for (int s = 0; s < S; ++s) nh[tt][s] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      floatx4 wa;
#pragma unroll
      for (int r = 0; r < 4; ++r) wa[r] = Wj[(long)(16 * kt + 4 * g + r) * W + 16 * rt + c];
#pragma unroll
      for (int tt = 0; tt < TH; ++tt) {
        const int t = h * TH + tt;
        floatx4 b4[S];
#pragma unroll
        for (int s = 0; s < S; ++s)
          b4[s] = *reinterpret_cast<const floatx4*>(zbp + (t * S + s) * PLANE + c * LDH + 16 * kt + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int s = 0; s < S; ++s) nh[tt][s] = mfma4(wa[r], b4[s][r], nh[tt][s]);
      }
    }
#pragma unroll
    for (int tt = 0; tt < TH; ++tt)
#pragma unroll
      for (int s = 0; s < S; ++s) hb[h][tt][s] = nh[tt][s];
  };

  using A_ = std::integral_constant<int, 0>;
  using B_ = std::integral_constant<int, 1>;
  using MID = std::integral_constant<bool, false>;
  using LAST = std::integral_constant<bool, true>;
  // One half-step: M of one half and V of the other.  The two waves sharing a SIMD
  // (w and w+4) take them in opposite orders, so while one issues the MFMA chain the
  // other runs its VALU work; a scheduling barrier keeps each wave's two parts apart
  // (their register states never coexist).
  // order 1: waves w, w+4 opposite; 2: waves 2k, 2k+1 opposite; 3: every wave M first
  const bool m_first = order == 3 ? true : (order == 2 ? (wave & 1) == 0 : (wave & 4) == 0);
  auto half_step = [&](auto HM, auto HV, auto LASTC, int jm, int jv) __attribute__((always_inline)) {
    if (m_first) {
      M(HM, jm);
      __builtin_amdgcn_sched_barrier(0);
      V(HV, LASTC, jv);
    } else {
      V(HV, LASTC, jv);
      __builtin_amdgcn_sched_barrier(0);
      M(HM, jm);
    }
  };
  // (the host launches this kernel for L >= 1 only)
  V(A_{}, MID{}, L);
  __syncthreads();
  for (int j = L; j >= 2; --j) {
    half_step(A_{}, B_{}, MID{}, j, j);
    __syncthreads();
    half_step(B_{}, A_{}, MID{}, j, j - 1);
    __syncthreads();
  }
  half_step(A_{}, B_{}, MID{}, 1, 1);
  __syncthreads();
  half_step(B_{}, A_{}, LAST{}, 1, 0);
  V(B_{}, LAST{}, 0);
}

template <int NT, int S, bool LAP, int T>
int launch_bwd_pipe_t(const float* x, int N, int din, int dout, int L, const float* prm, const float* act,
                      const float* gy, const float* gdy, const float* glap, float* part, long P, hipStream_t st,
                      int order) {
  constexpr size_t lds = bwd_split_lds_bytes<NT, S, T>();
  if constexpr (lds > kLdsMax || NT > 8 || T % 2 != 0) {
    return INSR_EINVAL;
  } else if (L < 1) {
    return launch_bwd_split_t<NT, S, LAP, T>(x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st);
  } else {
    const int nb = ((N + 15) / 16 + T - 1) / T;
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)jet_bwd_pipe<NT, S, LAP, T>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr_set = true;
    }
    hipLaunchKernelGGL((jet_bwd_pipe<NT, S, LAP, T>), dim3(nb), dim3(SplitGeo<NT>::THREADS), lds, st, x, N, din,
                       dout, L, prm, act, gy, gdy, glap, part, P, order);
    return (int)hipGetLastError();
  }
}

}  // namespace insr
