// jet_x6r.hpp -- the resident-dW backward of W = 128 SIRENs (jet_bwd_x6r): ONE launch walks
// every tile of the batch in a persistent per-CU loop and keeps the weight gradients of ALL
// hidden layers in the waves' registers from the first tile to the last, so the saved
// streams are read once and nothing per tile (no z̄, no dW partial) goes to HBM.
//
// Why (round-3 profiles, fluid2Dtlgn): the two-kernel path (jet_x6w.hpp) moves ~700 MB per
// Laplacian backward at 16,708 points -- the saved streams read twice (propagation kernel and
// dW GEMM) and z̄ written and read once -- and the fused tile-split backward (jet_x6.hpp) writes
// one full partial-gradient row per 5-tile block (209 x 266 KB) that a second kernel re-reads.
// Here: block b of nb (nb = CUs) takes tiles [b T / nb, (b + 1) T / nb), TS at a time (a
// "step": 2 tiles for value jets, so one dW K-chunk is 32 points; 1 tile otherwise); per step,
// layer j = L .. 1: sine reverse, z̄_j and h_{j-1} split into bf16 planes in LDS, then
//   dW_j += z̄_j h_{j-1}^T   (MFMA into dacc[j - 1]: 32 rows x 128 columns per wave)
//   h̄_{j-1} = W_j^T z̄_j    (MFMA, A from the pre-split W^T planes, next fragment prefetched)
// The biases, the first layer and the output layer (~1.4 K floats) accumulate in LDS (one owner
// lane per entry: a fixed order).  At the end the block writes its dW (L W^2 floats) and its
// compact row once; reduce_dw_kernel (jet_x6w.hpp) sums the nb partials in a fixed order.
// Traffic per launch: saved streams once + nb (L W^2 + compact) floats written and re-read.
//
// Registers: the block is 8 waves (two per SIMD, 256 registers per lane); wave w owns row tile w
// (16 rows) of every layer.  Its dW accumulators, L x 8 floatx4 = 128 registers at L = 4, stay
// in registers across the whole tile loop; the other 128 hold the propagation state.  The saved
// streams of layer j - 1 are loaded one layer ahead (value jets; the Laplacian state has no
// registers to spare), every W^T fragment one fragment ahead, the first one under the dW MFMAs.
// (4-wave blocks with 32 rows per wave and the dW in AGPRs -- one wave per SIMD -- measured
// slower at every size: RPW = 2, not instantiated.)  The partials are stored in fragment order.
// Reference semantics: loss.backward() (base/baseModel.py:73-78) through the jets of
// base/diff_ops.py:44-82 -- the math of jet_x6.hpp / jet_x6w.hpp, another summation order.
#pragma once
#include <type_traits>

#include "jet_x6w.hpp"

namespace insr {

constexpr int kX6rSmallMax = 1412;  // compact floats for W = 128, d_in, d_out <= 3, L <= 4 (16-B multiple)

template <int S>
constexpr int x6r_ts() { return S == 1 ? 2 : 1; }  // tiles per step

template <int NQ, int S>
constexpr size_t x6r_lds_bytes() {
  using BG = X6BwdGeo<NQ, 8>;
  return (size_t)x6r_ts<S>() * S * (BG::ZSET + BG::HSET) * 2 + (size_t)kX6rSmallMax * sizeof(float);
}

// h-stream s of a sine layer from sin / cos and the derivative z-streams held in registers
template <int S, bool LAP>
__device__ __forceinline__ floatx4 x6r_h(int s, const floatx4 (&zk)[S > 1 ? S - 1 : 1], const floatx4& sn,
                                         const floatx4& cs) {
  if constexpr (S == 1) {
    return sn;
  } else {
    return h_from_regs<S, LAP>(s, zk, sn, cs);
  }
}

template <int NQ, int S, bool LAP, int L, int RPW>
__global__ __launch_bounds__(512 / RPW, 1) void jet_bwd_x6r(const float* __restrict__ x, int N, int din, int dout,
                                                      const float* __restrict__ prm, const float* __restrict__ act,
                                                      const float* __restrict__ gy, const float* __restrict__ gdy,
                                                      const float* __restrict__ glap, float* __restrict__ dpart,
                                                      float* __restrict__ small, long Ps, int nb) {
  constexpr int NT = 8, W = 128, KC = 4, TB = 512 / RPW;  // 8 / RPW waves
  constexpr int TS = x6r_ts<S>();      // tiles per step
  constexpr int NSET = TS * S;          // 16-point sets of a step (set u = t S + s)
  constexpr int NCH = (NSET + 1) / 2;   // 32-deep K chunks of the step's dW
  constexpr bool PF = S <= 2;           // saved streams loaded one layer ahead
  using BG = X6BwdGeo<NQ, NT>;
  constexpr int LDB = BG::ZROW, ZPLANE = BG::ZPLANE, ZSET = BG::ZSET, HPLANE = BG::HPLANE, HSET = BG::HSET;
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  constexpr int ZK = S > 1 ? S - 1 : 1;
  extern __shared__ __attribute__((aligned(16))) float lds_f[];
  unsigned short* Z = reinterpret_cast<unsigned short*>(lds_f);
  unsigned short* H = Z + NSET * ZSET;
  float* sacc = reinterpret_cast<float*>(H + NSET * HSET);  // compact accumulators (Ps floats)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int rt0 = wave * RPW;  // this wave's row tiles: propagation outputs and dW rows
  const int ntiles = ((N + 63) / 64) * 4;
  const int tiles = (N + 15) / 16;
  const int t0 = (int)((long)blockIdx.x * tiles / nb), t1 = (int)((long)(blockIdx.x + 1) * tiles / nb);
  const long sb = (long)W * din + W;   // compact offset of b_1 (small_count layout, jet_x6w.hpp)
  const long so = sb + (long)L * W;    // compact offset of W_out
  const u32x4* wsp = wsp_base(prm, din, dout, L, W);
  const float* Wo = prm + out_off(din, W, L);
  for (int i = threadIdx.x; i < Ps; i += TB) sacc[i] = 0.f;

  floatx4 dacc[L][RPW][NT];
#pragma unroll
  for (int j = 0; j < L; ++j)
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) dacc[j][i][ct] = floatx4{0.f, 0.f, 0.f, 0.f};

  // raw saved streams of one layer for the step's tiles (slot t of a short step re-reads tile
  // tb: valid memory; its adjoints are zero, so it contributes nothing)
  auto fetch = [&](int layer, int tb, int cnt, floatx4(&zr)[TS][RPW][S]) {
#pragma unroll
    for (int t = 0; t < TS; ++t) {
      const float* base = act_base(act, layer, ntiles, tb + (t < cnt ? t : 0), S, NT);
      const bool l0 = l0_rebuilt(layer, L);  // the first layer's derivative streams: from W_0
#pragma unroll
      for (int i = 0; i < RPW; ++i)
#pragma unroll
        for (int s = 0; s < S; ++s) zr[t][i][s] = load_zs<NT, S, LAP>(base, s, rt0 + i, lane, l0, prm, din);
    }
  };
  // sin / cos and the derivative z-streams from the raw streams
  auto unpack = [&](const floatx4(&zr)[TS][RPW][S], floatx4(&s_)[TS][RPW], floatx4(&c_)[TS][RPW],
                    floatx4(&zk)[TS][RPW][ZK]) {
    float amax = 0.f;
#pragma unroll
    for (int t = 0; t < TS; ++t)
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
#pragma unroll
        for (int s = 1; s < S; ++s) zk[t][i][s - 1] = zr[t][i][s];
#pragma unroll
        for (int r = 0; r < 4; ++r) amax = fmaxf(amax, fabsf(OMEGA * zr[t][i][0][r]));
      }
    const bool big = wave_any_big(amax);
#pragma unroll
    for (int t = 0; t < TS; ++t)
#pragma unroll
      for (int i = 0; i < RPW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float sv, cv;
          if (big)
            sincosf(OMEGA * zr[t][i][0][r], &sv, &cv);
          else
            sincos_fast(OMEGA * zr[t][i][0][r], sv, cv);
          s_[t][i][r] = sv;
          c_[t][i][r] = cv;
        }
  };
  __syncthreads();  // sacc zeroed

  for (int tb = t0; tb < t1; tb += TS) {
    const int cnt = t1 - tb < TS ? t1 - tb : TS;
    auto adjoint = [&](int t, int s, int o) -> float {
      const int p = (tb + t) * 16 + c;
      if (t >= cnt || p >= N) return 0.f;
      if (s == 0) return gy ? gy[(long)p * dout + o] : 0.f;
      if (LAP && s == S - 1) return glap ? glap[(long)p * dout + o] : 0.f;
      return gdy ? gdy[((long)p * dout + o) * din + (s - 1)] : 0.f;
    };
    floatx4 sn[TS][RPW], cs[TS][RPW], zk[TS][RPW][ZK];
    floatx4 zr[TS][RPW][S];  // the next layer's raw streams (PF: one layer ahead)
    fetch(L, tb, cnt, zr);
    unpack(zr, sn, cs, zk);
    if constexpr (PF) fetch(L - 1, tb, cnt, zr);

    // ---- output layer (exact fp32 VALU): hb = W_out^T g, dW_out / db_out into the compact row ----
    floatx4 hb[TS][RPW][S];
#pragma unroll
    for (int t = 0; t < TS; ++t)
#pragma unroll
      for (int i = 0; i < RPW; ++i)
#pragma unroll
        for (int s = 0; s < S; ++s) hb[t][i][s] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int o = 0; o < dout; ++o) {
      float ga[TS][S];
#pragma unroll
      for (int t = 0; t < TS; ++t)
#pragma unroll
        for (int s = 0; s < S; ++s) ga[t][s] = adjoint(t, s, o);
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        const floatx4 w4 = *reinterpret_cast<const floatx4*>(Wo + (o * W + 16 * (rt0 + i) + 4 * g));
        floatx4 acc4 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < TS; ++t)
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const floatx4 hs = x6r_h<S, LAP>(s, zk[t][i], sn[t][i], cs[t][i]);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              acc4[r] = fmaf(ga[t][s], hs[r], acc4[r]);
              hb[t][i][s][r] = fmaf(w4[r], ga[t][s], hb[t][i][s][r]);
            }
          }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = sum16(acc4[r]);
          if (c == 0) sacc[so + (long)o * W + 16 * (rt0 + i) + 4 * g + r] += v;
        }
      }
      if (wave == 0) {
        float gsum = 0.f;
#pragma unroll
        for (int t = 0; t < TS; ++t) gsum += (g == 0) ? ga[t][0] : 0.f;
        const float v = sum16(gsum);
        if (lane == 0) sacc[so + (long)dout * W + o] += v;
      }
    }

    // ---- hidden layers j = L .. 1, each a compile-time j (dacc[j - 1] stays in registers) ----
    auto layer = [&](auto jc) {
      constexpr int j = decltype(jc)::value;
      // the W^T planes through an opaque pointer: their loads are step-invariant, and hoisting
      // them out of the tile loop would pin L x KC fragments in registers
      const u32x4* wsl = wsp;
      asm volatile("" : "+s"(wsl));
#pragma unroll
      for (int t = 0; t < TS; ++t)
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
          floatx4 zs[S];
          zs[0] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 1; s < S; ++s) zs[s] = zk[t][i][s - 1];
          sine_rev<S, LAP>(hb[t][i], zs, sn[t][i], cs[t][i]);  // hb = z̄_j
        }
#pragma unroll
      for (int i = 0; i < RPW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float bsum = 0.f;
#pragma unroll
          for (int t = 0; t < TS; ++t) bsum += hb[t][i][0][r];
          const float v = sum16(bsum);
          if (c == 0) sacc[sb + (long)(j - 1) * W + 16 * (rt0 + i) + 4 * g + r] += v;
        }
      floatx4 snp[TS][RPW], csp[TS][RPW], zkp[TS][RPW][ZK];
      if constexpr (!PF) fetch(j - 1, tb, cnt, zr);
      unpack(zr, snp, csp, zkp);
      if constexpr (PF) {
        if (j >= 2) fetch(j - 2, tb, cnt, zr);  // one layer ahead, in flight through this layer's MFMAs
      }
      __syncthreads();  // the previous layer's / step's LDS readers are done
#pragma unroll
      for (int t = 0; t < TS; ++t)
#pragma unroll
        for (int i = 0; i < RPW; ++i)
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const int u = t * S + s;
            lds_put4<NQ, ZPLANE>(Z + u * ZSET + c * LDB + 16 * (rt0 + i) + 4 * g, hb[t][i][s][0], hb[t][i][s][1],
                                 hb[t][i][s][2], hb[t][i][s][3]);
            put_neuron_major<NQ, HPLANE>(H + u * HSET, x6r_h<S, LAP>(s, zkp[t][i], snp[t][i], csp[t][i]),
                                         16 * (rt0 + i) + 4 * g, c);
          }
      __syncthreads();
      // the propagation's first W^T fragment is issued here: its L2 latency runs under the dW MFMAs
      FragQ<NQ> wn = wsp_frag<NQ, NT>(wsl, L, 1, j, rt0, 0, lane);
      // dW_j rows 16 rt + c (A: z̄ column reads of the point-major Z sets), columns m (B: H)
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int u = 2 * ch + (g >> 1);
        const bool live = u < NSET;
        const int p0 = 8 * (g & 1);
        FragQ<NQ> af[RPW];
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
          const unsigned short* pa = Z + (live ? u : 0) * ZSET + (p0 + (c >> 2)) * LDB + 16 * (rt0 + i) + 4 * (c & 3);
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const v4s lo = ds_read_tr16(pa + q * ZPLANE);
            const v4s hi = ds_read_tr16(pa + q * ZPLANE + 4 * LDB);
            const u32x2 wl = __builtin_bit_cast(u32x2, lo), wh = __builtin_bit_cast(u32x2, hi);
            af[i].q[q] = live ? u32x4{wl[0], wl[1], wh[0], wh[1]} : u32x4{0u, 0u, 0u, 0u};
          }
        }
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
          const FragQ<NQ> bf = lds_frag<NQ, HPLANE>(H + (live ? u : 0) * HSET + (16 * ct + c) * 16 + p0);
#pragma unroll
          for (int i = 0; i < RPW; ++i) dacc[j - 1][i][ct] = mfma_q<NQ>(af[i], bf, dacc[j - 1][i][ct]);
          X6_SCHED_FENCE();
        }
      }
      // propagation: h̄_{j-1}[m] = sum_n W_j[n][m] z̄_j[n] (A = W^T fragments, B = Z rows); the
      // fragments in (row tile, K chunk) order, each prefetched one ahead
      floatx4 nh[TS][RPW][S];
#pragma unroll
      for (int t = 0; t < TS; ++t)
#pragma unroll
        for (int i = 0; i < RPW; ++i)
#pragma unroll
          for (int s = 0; s < S; ++s) nh[t][i][s] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int f = 0; f < RPW * KC; ++f) {
        const int i = f / KC, kc = f % KC;
        const FragQ<NQ> wt = wn;
        if (f + 1 < RPW * KC) wn = wsp_frag<NQ, NT>(wsl, L, 1, j, rt0 + (f + 1) / KC, (f + 1) % KC, lane);
#pragma unroll
        for (int t = 0; t < TS; ++t)
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const FragQ<NQ> bf = lds_frag<NQ, ZPLANE>(Z + (t * S + s) * ZSET + c * LDB + 32 * kc + 8 * g);
            nh[t][i][s] = mfma_q<NQ>(wt, bf, nh[t][i][s]);
            X6_SCHED_FENCE();
          }
      }
#pragma unroll
      for (int t = 0; t < TS; ++t)
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
#pragma unroll
          for (int s = 0; s < S; ++s) hb[t][i][s] = nh[t][i][s];
          sn[t][i] = snp[t][i];
          cs[t][i] = csp[t][i];
#pragma unroll
          for (int s = 0; s < ZK; ++s) zk[t][i][s] = zkp[t][i][s];
        }
    };
    if constexpr (L >= 4) layer(std::integral_constant<int, 4>{});
    if constexpr (L >= 3) layer(std::integral_constant<int, 3>{});
    if constexpr (L >= 2) layer(std::integral_constant<int, 2>{});
    layer(std::integral_constant<int, 1>{});

    // ---- first layer (K = d_in: exact fp32 VALU) ----
    float xk[TS][3];
#pragma unroll
    for (int t = 0; t < TS; ++t) {
      const int p = (tb + t) * 16 + c;
      for (int k = 0; k < 3; ++k) xk[t][k] = (t < cnt && p < N && k < din) ? x[(long)p * din + k] : 0.f;
    }
#pragma unroll
    for (int t = 0; t < TS; ++t)
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        floatx4 zs[S];
        zs[0] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 1; s < S; ++s) zs[s] = zk[t][i][s - 1];
        sine_rev<S, LAP>(hb[t][i], zs, sn[t][i], cs[t][i]);  // hb = z̄_0
      }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float bsum = 0.f;
#pragma unroll
        for (int t = 0; t < TS; ++t) bsum += hb[t][i][0][r];
        const float v = sum16(bsum);
        if (c == 0) sacc[(long)W * din + 16 * (rt0 + i) + 4 * g + r] += v;
      }
      for (int k = 0; k < din; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = 0.f;
#pragma unroll
          for (int t = 0; t < TS; ++t) {
            v = fmaf(hb[t][i][0][r], xk[t][k], v);
            if (k < NTAN) v += hb[t][i][1 + k][r];
          }
          v = sum16(v);
          if (c == 0) sacc[(long)(16 * (rt0 + i) + 4 * g + r) * din + k] += v;
        }
    }
  }

  // ---- the block's partials: dW of every hidden layer in fragment order (one 1 KiB wave store per
  // accumulator; reduce_dw_kernel frag = 1 scatters the sums), then the compact row ----
#pragma unroll
  for (int jl = 0; jl < L; ++jl) {
    floatx4* out = reinterpret_cast<floatx4*>(dpart + ((long)jl * nb + blockIdx.x) * W * W);
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) out[((rt0 + i) * NT + ct) * 64 + lane] = dacc[jl][i][ct];
  }
  __syncthreads();  // every owner lane's last compact update
  for (int i = threadIdx.x; i < Ps; i += TB) small[(long)blockIdx.x * Ps + i] = sacc[i];
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
inline int x6r_blocks(long n) {
  const int cus = device_cus();
  const long tiles = (n + 15) / 16;
  if (tiles <= cus) return (int)(tiles > 0 ? tiles : 1);
  const long per = (tiles + cus - 1) / cus;  // balanced: fewest blocks at the same tiles per block (jet_fb.hpp)
  return (int)((tiles + per - 1) / per);
}

// workspace floats: dW partials [layer][block][W^2] | compact rows [block][Ps]
inline long x6r_work_floats(long n, int din, int dout, int L) {
  const long nb = x6r_blocks(n);
  return (long)L * nb * 128 * 128 + nb * small_count(din, dout, L, 128);
}

template <int NQ, int S, bool LAP, int L, int RPW>
int resident_bwd_t(const float* x, int N, int din, int dout, const float* prm, const float* act, const float* gy,
                   const float* gdy, const float* glap, float* work, float* grad, int accumulate, hipStream_t st) {
  constexpr int W = 128;
  const int nb = x6r_blocks(N);
  const long Ps = small_count(din, dout, L, W);
  if (Ps > kX6rSmallMax) return INSR_EINVAL;
  float* dpart = work;
  float* small = dpart + (long)L * nb * W * W;
  constexpr size_t lds = x6r_lds_bytes<NQ, S>();
  static_assert(lds <= 163840, "LDS");
  static_assert(L >= 1 && L <= 4, "resident dW: 1..4 hidden layers");
  static const bool attr = ((void)hipFuncSetAttribute((const void*)jet_bwd_x6r<NQ, S, LAP, L, RPW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds), true);  // once per instantiation (thread-safe static init)
  (void)attr;
  hipLaunchKernelGGL((jet_bwd_x6r<NQ, S, LAP, L, RPW>), dim3(nb), dim3(512 / RPW), lds, st, x, N, din, dout, prm, act, gy, gdy,
                     glap, dpart, small, Ps, nb);
  const int grad16 = (((uintptr_t)(grad + hidden_off(din, W, 1))) & 15) == 0 ? 1 : 0;
  const int wq = (W * W / 4 + 63) / 64;
  const int rows_x = (int)((Ps + 63) / 64);
  hipLaunchKernelGGL(reduce_dw_kernel, dim3((unsigned)(wq > rows_x ? wq : rows_x), L + 1), dim3(512), 0, st, dpart, nb,
                     din, W, grad, accumulate, grad16, 1, L, small, nb, Ps, dout, 1, nb, AdamArgs{});
  return (int)hipGetLastError();
}

}  // namespace insr
