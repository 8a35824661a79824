// jet_x6w.hip -- the backward of WIDE SIRENs (W = 256: elasticity3Dbunny, SIREN 5x256)
// as two split-bf16 ("x6", jet_x6.hpp) kernels instead of one:
//
//   jet_bwd_x6p   per 16-point tile, the reverse sweep with ADJOINT PROPAGATION only:
//                 h̄_{j-1} = W_j^T z̄_j on the matrix cores; it stores z̄_j (j >= 1) to HBM
//                 in the saved-activation layout and writes a COMPACT partial row per
//                 tile: the gradients of the first layer, every bias and the output layer.
//   dw_x6         dW_j = sum over points p and streams s of z̄_j[p,s,:] (x) h_{j-1}[p,s,:]
//                 for the hidden layers, as a split-K GEMM over K = points x streams: z̄
//                 from HBM, h rebuilt from the forward's saved z (sin/cos + jet streams),
//                 both split to bf16 planes in LDS; one partial W x W per (layer, K slice).
//
// Why: the fused tile-split backward keeps each wave's dW rows for all W columns in
// registers (W = 256: 128 VGPRs) next to the propagation state, which does not fit for
// the x6 path, and it writes one FULL partial-gradient row (330,755 floats = 1.3 MB) per
// 16 points: 21.7 GB written and read again at 262,144 points.  Here the hidden-layer
// gradient is a GEMM with K = N x S (one partial per K slice: ~100 per layer) and the
// per-tile rows shrink to the 3,075 non-hidden parameters.
//
// Reference semantics: loss.backward() of base/baseModel.py:73-78 through the jets of
// base/diff_ops.py:44-82 (the same math as jet_split.hpp / jet_x6.hpp).
#include "jet_x6.hpp"
#include "optim.hpp"

// the wide path is compiled once per precision TU: jet_x6w.hip (NQ = 3) and jet_bfw.hip
// (NQ = 1, 2) include this file with INSR_WIDE_NQ set
#ifndef INSR_WIDE_NQ_DEFS
#define INSR_WIDE_NQ_DEFS

namespace insr {


// compact partial row of the wide path: [W0 (W din) | b0 (W) | b_1 .. b_L (L W) | Wout (dout W) | bout]
__host__ __device__ inline long small_count(int din, int dout, int L, int W) {
  return (long)W * din + W + (long)L * W + (long)dout * W + dout;
}

// ---------------------------------------------------------------------------------------
// the pre-split weight planes (INSR_MODE_WSPLIT, jet_common.hpp wsplit_offset): one thread per
// (orientation o, layer j - 1, fragment (rt, kc), lane (g, c)): the 8 weights
//   o = 0: W_j[16 rt + c][32 kc + 8 g + 0..7]   (forward A operand, contiguous)
//   o = 1: W_j[32 kc + 8 g + 0..7][16 rt + c]   (backward A operand = W_j^T rows)
// split in three bf16 terms (split_frag<3>); kernels of NQ < 3 read the first NQ terms;
//   o = 2: the o = 0 weights times 2^8 in two fp16 terms (split_frag<4>: INSR_PREC_F16X3),
//          after the two bf16 orientations; o = 3: the o = 1 weights likewise (the f16x3 backward)
// ---------------------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(256) void wsplit_kernel(const float* __restrict__ prm, int din, int L,
                                                     u32x4* __restrict__ out, unsigned* __restrict__ status) {
  constexpr int W = 16 * NT, KC = NT / 2, NF = NT * KC;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = (int)(gid & 63), g = lane >> 4, c = lane & 15;
  const long fa = gid >> 6;  // (o, layer, frag)
  if (fa >= 4L * L * NF) return;
  const int o = (int)(fa / ((long)L * NF));
  const long f = fa % ((long)L * NF);
  const int j = 1 + (int)(f / NF), rt = (int)((f % NF) / KC), kc = (int)(f % KC);
  const float* Wj = prm + hidden_off(din, W, j);
  floatx4 v0, v1;
  if (o == 0 || o == 2) {
    v0 = *reinterpret_cast<const floatx4*>(Wj + (16 * rt + c) * W + 32 * kc + 8 * g);
    v1 = *reinterpret_cast<const floatx4*>(Wj + (16 * rt + c) * W + 32 * kc + 8 * g + 4);
  } else {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      v0[jj] = Wj[(32 * kc + 8 * g + jj) * W + 16 * rt + c];
      v1[jj] = Wj[(32 * kc + 8 * g + 4 + jj) * W + 16 * rt + c];
    }
  }
  if (o >= 2) {  // fp16: o = 2 forward rows, o = 3 backward (W^T) rows
    float m = 0.f;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) m = fmaxf(m, fmaxf(fabsf(v0[jj]), fabsf(v1[jj])));
    if (!(m < kF16WMax)) {  // outside the planes' range (or NaN): flag it, keep the terms finite
      if (o == 2) atomicOr(status, 1u);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        v0[jj] = fminf(fmaxf(v0[jj], -kF16WMax), kF16WMax);
        v1[jj] = fminf(fmaxf(v1[jj], -kF16WMax), kF16WMax);
      }
    }
    const FragQ<4> h = split_frag<4>(v0 * kF16WScale, v1 * kF16WScale);
    u32x4* oh = out + (o == 2 ? 6L : 8L) * L * NF * 64;  // after both bf16 orientations (3 L W^2 floats)
    const long fh = f;
#pragma unroll
    for (int k = 0; k < 2; ++k) oh[(fh * 2 + k) * 64 + lane] = h.q[k];
    return;
  }
  const FragQ<3> q = split_frag<3>(v0, v1);
#pragma unroll
  for (int k = 0; k < 3; ++k) out[(fa * 3 + k) * 64 + lane] = q.q[k];
}

// ---------------------------------------------------------------------------------------
// kernel 1: propagation-only reverse sweep (one 16-point tile per block, 8 waves x 2 row tiles)
// ---------------------------------------------------------------------------------------
// W = 128: held to 128 VGPRs (4 waves per SIMD = two 8-wave blocks per CU; its 52 KB of LDS
// allow three) -- the one-tile sweep is latency-bound, a second resident block hides it
// (the f16x3 variant: INSR_F16_BWD_WAVES waves per SIMD, A/B builds only)
#ifndef INSR_F16_BWD_WAVES
#define INSR_F16_BWD_WAVES 4
#endif
template <int NQ, int NT>
constexpr int x6p_min_waves() { return NT == 8 ? (NQ == 4 ? INSR_F16_BWD_WAVES : 4) : 1; }

template <int NQ, int NT, int S, bool LAP>
__global__ __launch_bounds__(512, (x6p_min_waves<NQ, NT>())) void jet_bwd_x6p(const FbJobs J, int N, int din, int dout, int L,
                                                   const float* __restrict__ prm, float* __restrict__ adj,
                                                   float* __restrict__ part, long Ps, float* __restrict__ zmax) {
  constexpr int W = 16 * NT, RPW = NT / 8, KC = NT / 2;
  constexpr int LDB = W + 8, ZPLANE = 16 * LDB, ZSET = np_of<NQ>() * ZPLANE;
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  // NQ = 4 (INSR_BWD_F16_PROP): the propagation on the fp16 matrix cores -- W^T from the fp16
  // backward planes (x 2^8), z̄ scaled per tile by the power of two 2^e that maps the tile's largest
  // |z̄| (Laplacian stream x 16) into [2^14, 2^15), the product unscaled by 2^-(8 + e) (exact)
  extern __shared__ __attribute__((aligned(16))) float lds_f[];
  unsigned short* Z = reinterpret_cast<unsigned short*>(lds_f);  // [s][q][16 p][W + 8]
  float* zred = lds_f + S * ZSET / 2;                             // [2][3][8 waves]: tile maxima
  const int tiles_n = (N + 15) / 16;
  // f16 dW (zmax != NULL): zq [L][tiles][3] = this tile's max |z̄_j| over the value stream, the tangent
  // streams and the Laplacian stream (slot j - 1), then hq [L][tiles][8] = each wave's bound of the
  // Laplacian stream of h_j = w c q - w^2 s sum t^2, i.e. w |q| + w^2 sum t^2 (slot j, j < L), then
  // ht [L][tiles][8] = each wave's bound of h_j's tangent streams, w |t|
  float* zq = zmax;
  float* hq = zmax ? zmax + 3L * L * tiles_n : nullptr;
  float* ht = zmax ? hq + 8L * L * tiles_n : nullptr;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  // several jobs (round 6: e.g. an interior batch and its constraint bands from separate network calls):
  // block = tile of the launch (z̄, the compact rows and the maxima are laid out by it, over N = 16 x the
  // jobs' tiles); the job's points, adjoints and saved streams by its own tile lt
  const int ntiles = ((N + 63) / 64) * 4;
  const int tile = blockIdx.x;
  int jk = 0;
#pragma unroll
  for (int q = 1; q < kBwdJobs; ++q) jk += (q < J.njobs && tile >= J.tstart[q]) ? 1 : 0;
  const int lt = tile - J.tstart[jk], Nk = J.n[jk];
  const int ntk = ((Nk + 63) / 64) * 4;
  const float* __restrict__ x = J.x[jk];
  const float* __restrict__ act = J.act[jk];
  const float* __restrict__ gy = J.gy[jk];
  const float* __restrict__ gdy = J.gdy[jk];
  const float* __restrict__ glap = J.glap[jk];
  const int rt0 = wave * RPW;
  const int p = lt * 16 + c;
  const bool valid = p < Nk;
  float* mypart = part + (long)blockIdx.x * Ps;
  const long sb = (long)W * din + W;       // compact offset of b_1
  const long so = sb + (long)L * W;        // compact offset of Wout

  auto adjoint = [&](int s, int o) -> float {
    if (!valid) return 0.f;
    if (s == 0) return gy ? gy[(long)p * dout + o] : 0.f;
    if (LAP && s == S - 1) return glap ? glap[(long)p * dout + o] : 0.f;
    return gdy ? gdy[((long)p * dout + o) * din + (s - 1)] : 0.f;
  };
  auto load_sc = [&](int layer, floatx4(&s_)[RPW], floatx4(&c_)[RPW]) {
    const float* base = act_base(act, layer, ntk, lt, S, NT);
    floatx4 z[RPW];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      z[i] = *reinterpret_cast<const floatx4*>(base + ((rt0 + i) * 64 + lane) * 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) amax = fmaxf(amax, fabsf(OMEGA * z[i][r]));
    }
    const bool big = wave_any_big(amax);
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float sv, cv;
        if (big)
          sincosf(OMEGA * z[i][r], &sv, &cv);
        else
          sincos_fast(OMEGA * z[i][r], sv, cv);
        s_[i][r] = sv;
        c_[i][r] = cv;
      }
  };

  // ---- output layer (exact fp32 VALU) ----
  floatx4 sn[RPW], cs[RPW];
  load_sc(L, sn, cs);
  const float* Wo = prm + out_off(din, W, L);
  floatx4 hb[RPW][S];
#pragma unroll
  for (int i = 0; i < RPW; ++i)
#pragma unroll
    for (int s = 0; s < S; ++s) hb[i][s] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float* baseL = act_base(act, L, ntk, lt, S, NT);
  for (int o = 0; o < dout; ++o) {
    float ga[S];
#pragma unroll
    for (int s = 0; s < S; ++s) ga[s] = adjoint(s, o);
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int rt = rt0 + i;
      const floatx4 w4 = *reinterpret_cast<const floatx4*>(Wo + (o * W + 16 * rt + 4 * g));
      floatx4 acc4 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const floatx4 hs = h_stream<NT, S, LAP>(baseL, s, rt, lane, sn[i], cs[i]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc4[r] = fmaf(ga[s], hs[r], acc4[r]);
          hb[i][s][r] = fmaf(w4[r], ga[s], hb[i][s][r]);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = sum16(acc4[r]);
        if (c == 0) mypart[so + (long)o * W + 16 * rt + 4 * g + r] = v;
      }
    }
    if (wave == 0) {
      float v = sum16(g == 0 ? ga[0] : 0.f);
      if (lane == 0) mypart[so + (long)dout * W + o] = v;
    }
  }

  // ---- sine layers j = L .. 0 ----
  for (int j = L; j >= 0; --j) {
    const float* basej = act_base(act, j, ntk, lt, S, NT);
    float hl = 0.f, htb = 0.f;  // this wave's bounds of |h_j|'s Laplacian and tangent streams
    constexpr int NTAN = LAP ? S - 2 : S - 1;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      floatx4 zs[S];
#pragma unroll
      for (int s = 0; s < S; ++s)
        zs[s] = (s == 0) ? floatx4{0.f, 0.f, 0.f, 0.f}
                         : load_zs<NT, S, LAP>(basej, s, rt0 + i, lane, l0_rebuilt(j, L), prm, din);
      if (hq && j < L) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float t2 = 0.f;
#pragma unroll
          for (int k = 1; k <= NTAN; ++k) {
            t2 = fmaf(zs[k][r], zs[k][r], t2);
            htb = fmaxf(htb, fabsf(zs[k][r]));
          }
          if constexpr (LAP) hl = fmaxf(hl, fmaf(OMEGA, fabsf(zs[S - 1][r]), OMEGA2 * t2));
        }
      }
      sine_rev<S, LAP>(hb[i], zs, sn[i], cs[i]);  // hb = z̄_j
    }
    if (hq && j < L) {
      if constexpr (LAP) {
        hl = wave_max(hl);
        if (lane == 0) hq[((long)j * tiles_n + tile) * 8 + wave] = hl;
      }
      if constexpr (NTAN > 0) {
        htb = wave_max(htb) * OMEGA;
        if (lane == 0) ht[((long)j * tiles_n + tile) * 8 + wave] = htb;
      }
    }
    const long boff = (j == 0) ? (long)W * din : sb + (long)(j - 1) * W;
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = sum16(hb[i][0][r]);
        if (c == 0) mypart[boff + 16 * (rt0 + i) + 4 * g + r] = v;
      }
    if (j == 0) {
      float xk[3];
      for (int k = 0; k < 3; ++k) xk[k] = (valid && k < din) ? x[(long)p * din + k] : 0.f;
#pragma unroll
      for (int i = 0; i < RPW; ++i)
        for (int k = 0; k < din; ++k)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = hb[i][0][r] * xk[k];
            if (k < NTAN) v += hb[i][1 + k][r];
            v = sum16(v);
            if (c == 0) mypart[(long)(16 * (rt0 + i) + 4 * g + r) * din + k] = v;
          }
      break;
    }
    // z̄_j -> HBM (layer slot j - 1), the A operand of dw_x6
    {
      float* ab = act_base(adj, j - 1, ntiles, tile, S, NT);
#pragma unroll
      for (int i = 0; i < RPW; ++i)
#pragma unroll
        for (int s = 0; s < S; ++s) *reinterpret_cast<floatx4*>(ab + ((s * NT + rt0 + i) * 64 + lane) * 4) = hb[i][s];
    }
    if (zmax || NQ == 4) {  // this wave's max |z̄_j| over the value, tangent and Laplacian streams
      float mv = 0.f, mt = 0.f, ml = 0.f;
#pragma unroll
      for (int i = 0; i < RPW; ++i)
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (LAP && s == S - 1)
              ml = fmaxf(ml, fabsf(hb[i][s][r]));
            else if (s == 0)
              mv = fmaxf(mv, fabsf(hb[i][s][r]));
            else
              mt = fmaxf(mt, fabsf(hb[i][s][r]));
          }
      mv = wave_max(mv);
      if constexpr (S > 1) mt = wave_max(mt);
      if constexpr (LAP) ml = wave_max(ml);
      if (lane == 0) {  // two slots: layer j - 1 writes the other
        zred[((j & 1) * 3) * 8 + wave] = mv;
        zred[((j & 1) * 3 + 1) * 8 + wave] = mt;
        zred[((j & 1) * 3 + 2) * 8 + wave] = ml;
      }
    }
    __syncthreads();  // the previous layer's readers of Z are done
    // NQ = 4: the tile's adjoint scales 2^e (value / tangent streams, Laplacian stream: each its own
    // accumulators here) and the products' unscales 2^-(8 + e)
    float zso = 1.f, zsl = 1.f, zuo = 1.f, zul = 1.f;
    if constexpr (NQ == 4) {
      float mo = fmaxf(zred[((j & 1) * 3) * 8], zred[((j & 1) * 3 + 1) * 8]), ml = zred[((j & 1) * 3 + 2) * 8];
#pragma unroll
      for (int w = 1; w < 8; ++w) {
        mo = fmaxf(mo, fmaxf(zred[((j & 1) * 3) * 8 + w], zred[((j & 1) * 3 + 1) * 8 + w]));
        ml = fmaxf(ml, zred[((j & 1) * 3 + 2) * 8 + w]);
      }
      const int eo = f16_exp_for(mo), el = f16_exp_for(ml);
      zso = ldexpf(1.f, eo);
      zuo = ldexpf(1.f, -eo) / kF16WScale;
      zsl = ldexpf(1.f, el);
      zul = ldexpf(1.f, -el) / kF16WScale;
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const float f = (LAP && s == S - 1) ? zsl : zso;
        lds_put4<NQ, ZPLANE>(Z + s * ZSET + c * LDB + 16 * (rt0 + i) + 4 * g, hb[i][s][0] * f, hb[i][s][1] * f,
                             hb[i][s][2] * f, hb[i][s][3] * f);
      }
    __syncthreads();
    if (zq && threadIdx.x == 0) {
      float m3[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        m3[k] = zred[((j & 1) * 3 + k) * 8];
#pragma unroll
        for (int w = 1; w < 8; ++w) m3[k] = fmaxf(m3[k], zred[((j & 1) * 3 + k) * 8 + w]);
        zq[((long)(j - 1) * tiles_n + tile) * 3 + k] = m3[k];
      }
    }
    // propagation: h̄_{j-1}[m] = sum_n W_j[n][m] z̄_j[n]; A = W^T rows m of this wave (pre-split
    // planes, orientation 1: NQ b128 loads per fragment), B = Z rows (one b128 per plane)
    const u32x4* wsp = wsp_base(prm, din, dout, L, W);
    floatx4 nh[RPW][S];
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int s = 0; s < S; ++s) nh[i][s] = floatx4{0.f, 0.f, 0.f, 0.f};
    FragQ<NQ> wn[RPW];
    auto load_wt = [&](int kc) {
#pragma unroll
      for (int i = 0; i < RPW; ++i) wn[i] = wsp_frag<NQ, NT>(wsp, L, 1, j, rt0 + i, kc, lane);
    };
    load_wt(0);
#pragma unroll 1
    for (int kc = 0; kc < KC; ++kc) {
      FragQ<NQ> wt[RPW];
#pragma unroll
      for (int i = 0; i < RPW; ++i) wt[i] = wn[i];
      if (kc + 1 < KC) load_wt(kc + 1);  // L2-resident planes, in flight during this chunk's MFMAs
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const FragQ<NQ> bf = lds_frag<NQ, ZPLANE>(Z + s * ZSET + c * LDB + 32 * kc + 8 * g);
#pragma unroll
        for (int i = 0; i < RPW; ++i) nh[i][s] = mfma_q<NQ>(wt[i], bf, nh[i][s]);
        X6_SCHED_FENCE();  // keep the next stream's B reads from being hoisted (register budget)
      }
    }
    load_sc(j - 1, sn, cs);  // sin/cos of layer j-1 for the next sine reverse
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int s = 0; s < S; ++s) hb[i][s] = (NQ == 4) ? nh[i][s] * ((LAP && s == S - 1) ? zul : zuo) : nh[i][s];
  }
}

// ---------------------------------------------------------------------------------------
// kernel 2: hidden-layer weight gradients, split-K GEMM on the x6 matrix cores
//   block (slice, layer j = blockIdx.y + 1): 8 waves; wave w owns dW rows n in row tiles
//   {2w, 2w + 1} x all 16 column tiles (128 accumulator VGPRs).  K is walked in chunks of
//   two (tile, stream) units = 32 = one v_mfma_f32_16x16x32_bf16 k-step.  LDS images:
//   A = z̄ [q][n][k], B = h [q][m][k] (k minor, rows padded to 40: conflict-free b128 reads);
//   the loaders pack two adjacent points per u32 (DPP lane swap) and split each value once.
// ---------------------------------------------------------------------------------------
constexpr int kDwKR = 40;  // k row (32 + 8 pad) in bf16 elements
template <int NT>
constexpr int dw_plane() { return 16 * NT * kDwKR; }  // one plane (bf16 elements)
template <int NQ, int NT>
constexpr size_t dw_lds() { return (size_t)2 * np_of<NQ>() * dw_plane<NT>() * 2; }  // A + B, np_of<NQ> planes each

__device__ __forceinline__ float swap1(float v) {  // value of lane ^ 1 (quad_perm 1,0,3,2)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
}

// write one granule (4 neurons 4g..4g+3 of row tile rt, point c) as point pairs into the
// k-minor planes: even lanes write neurons r = 0, 1 of points (c, c + 1), odd lanes r = 2, 3
// of points (c - 1, c)
template <int NQ, int NT>
__device__ __forceinline__ void dw_put(unsigned short* P, const floatx4& v, int rt, int ul, int lane) {
  constexpr int kDwPL = dw_plane<NT>();
  const int g = lane >> 4, c = lane & 15, odd = c & 1;
  const float r0 = swap1(odd ? v[0] : v[2]);
  const float r1 = swap1(odd ? v[1] : v[3]);
  const float a0 = odd ? r0 : v[0], b0 = odd ? v[2] : r0;
  const float a1 = odd ? r1 : v[1], b1 = odd ? v[3] : r1;
  const int n0 = 16 * rt + 4 * g + (odd ? 2 : 0);
  const int k = 16 * ul + (c & ~1);
  unsigned u[np_of<NQ>()];
  splitq<NQ>(a0, b0, u);
  unsigned* q0 = reinterpret_cast<unsigned*>(P + n0 * kDwKR + k);
#pragma unroll
  for (int q = 0; q < np_of<NQ>(); ++q) q0[q * (kDwPL / 2)] = u[q];
  splitq<NQ>(a1, b1, u);
  unsigned* q1 = reinterpret_cast<unsigned*>(P + (n0 + 1) * kDwKR + k);
#pragma unroll
  for (int q = 0; q < np_of<NQ>(); ++q) q1[q * (kDwPL / 2)] = u[q];
}

// first level of the compact-row reduction, 8 waves: column block bx of out row by (of nby)
// = the fixed-order sum of part rows [nb by / nby, nb (by+1) / nby).  red: 512 floats of LDS.
__device__ __forceinline__ void rows_level1(const float* __restrict__ part, int nb, long count, float* __restrict__ out,
                                            int bx, int by, int nby, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long i = (long)bx * 64 + lane;
  const int b0 = (int)((long)nb * by / nby), b1 = (int)((long)nb * (by + 1) / nby);
  float acc = 0.f;
  if (i < count) {
    int b = b0 + w;
    for (; b + 56 < b1; b += 64) {  // 8 independent loads in flight per thread
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long)(b + 8 * u) * count + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; b < b1; b += 8) acc += part[(long)b * count + i];
  }
  red[w * 64 + lane] = acc;
  __syncthreads();
  if (w == 0 && i < count) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k * 64 + lane];
    out[(long)by * count + i] = t;
  }
}

// dW of hidden layer blockIdx.y + 1 over chunk slice blockIdx.x (y < L).  Planes y >= L carry
// the first level of the compact-row reduction (small -> rows, block id (y - L) KS + x), so it
// runs on the CUs the dW tail leaves idle instead of in a launch of its own.
// NQ = 4 (f16x3, the x6 backward's dW under INSR_BWD_F16_DW): fp16 has 11 significant bits but a
// narrow range, and neither an adjoint nor h's Laplacian stream has an a-priori scale, so each K
// slice takes powers of two from the propagation kernel's tile maxima (zq, hq): h's Laplacian stream
// x 2^eh (its bound's maximum into [2^14, 2^15)), value / tangent streams of h unscaled (|dh| <= w |t|),
// z̄ x 2^e on the value / tangent streams and x 2^(e - eh) on the Laplacian one, e mapping the larger
// of the two maxima into [2^14, 2^15) -- every product carries 2^e, undone on the partial (exact).
template <int NQ, int NT, int S, bool LAP>
__global__ __launch_bounds__(512, (NQ == 4 && NT == 8) ? INSR_F16_BWD_WAVES : 1) void dw_x6(int N, const FbJobs J, const float* __restrict__ adj,
                                             float* __restrict__ dpart, int KS, int L, const float* __restrict__ small,
                                             int tiles, long Ps, float* __restrict__ rows, int rs, int rows_x,
                                             const float* __restrict__ zmax, const float* __restrict__ w0, int din) {
  constexpr int W = 16 * NT, RT = NT / 8;  // RT: dW row tiles per wave
  constexpr int G = NT / 4;                   // granules per thread per chunk (2 units x NT row tiles / 8 waves)
  constexpr int kDwPL = dw_plane<NT>();
  extern __shared__ __attribute__((aligned(16))) float lds_f[];
  unsigned short* A = reinterpret_cast<unsigned short*>(lds_f);
  unsigned short* B = A + np_of<NQ>() * kDwPL;
  if ((int)blockIdx.y >= L) {
    const int rb = ((int)blockIdx.y - L) * KS + (int)blockIdx.x;
    if (rb < rows_x * rs) rows_level1(small, tiles, Ps, rows, rb % rows_x, rb / rows_x, rs, lds_f);
    return;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int j = blockIdx.y + 1;
  const bool l0 = l0_rebuilt(j - 1, L);  // h_0's derivative streams: rebuilt from W_0 (not saved)
  const int ntiles = ((N + 63) / 64) * 4;  // z̄: launch tiles (all jobs)
  const int units = ((N + 15) / 16) * S;
  // saved streams of launch tile t: its job's buffer at the job's own tile (t wave-uniform)
  auto abase = [&](int t) -> const float* {
    int k = 0;
#pragma unroll
    for (int q = 1; q < kBwdJobs; ++q) k += (q < J.njobs && t >= J.tstart[q]) ? 1 : 0;
    return act_base(J.act[k], j - 1, ((J.n[k] + 63) / 64) * 4, t - J.tstart[k], S, NT);
  };
  const int chunks = (units + 1) / 2;
  const int c0 = (int)((long)chunks * blockIdx.x / KS), c1 = (int)((long)chunks * (blockIdx.x + 1) / KS);
  // fp16 operand scales (NQ = 4): z̄ x asc (x ascl more on the Laplacian stream), h's Laplacian
  // stream x bscl, the partial x osc
  // h's tangent streams enter unscaled while their bound w |t| stays below 2^15 (the common case, as
  // before); a slice holding a larger bound scales them x 2^eht and the z̄ tangent streams x 2^-eht
  // (every product keeps 2^e); ascl / asct / bsct: those factors
  float asc = 1.f, ascl = 1.f, bscl = 1.f, osc = 1.f, asct = 1.f, bsct = 1.f;
  if constexpr (NQ == 4) {
    float mv = 0.f, mt = 0.f, ml = 0.f, mh = 0.f, mht = 0.f;
    if (c1 > c0) {
      const int ta = (2 * c0) / S, tb = min((2 * c1 - 1) / S, tiles - 1);
      const float* hq = zmax + 3L * L * tiles;
      const float* htq = hq + 8L * L * tiles;
      for (int t = ta + lane; t <= tb; t += 64) {
        mv = fmaxf(mv, zmax[((long)(j - 1) * tiles + t) * 3]);
        mt = fmaxf(mt, zmax[((long)(j - 1) * tiles + t) * 3 + 1]);
        ml = fmaxf(ml, zmax[((long)(j - 1) * tiles + t) * 3 + 2]);
      }
      for (int q = lane; q < (tb - ta + 1) * 8; q += 64) {
        if constexpr (LAP) mh = fmaxf(mh, hq[((long)(j - 1) * tiles + ta) * 8 + q]);
        if constexpr (S > 1) mht = fmaxf(mht, htq[((long)(j - 1) * tiles + ta) * 8 + q]);
      }
    }
    mv = wave_max(mv);
    mt = wave_max(mt);
    ml = wave_max(ml);
    mh = wave_max(mh);
    mht = wave_max(mht);
    const int eh = LAP ? f16_exp_for(mh) : 0;
    const int eht = mht >= 32768.f ? f16_exp_for(mht) : 0;
    const float bl = ldexpf(1.f, eh), bt = ldexpf(1.f, eht);
    const int e = f16_exp_for(fmaxf(mv, fmaxf(mt / bt, ml / bl)));
    asc = ldexpf(1.f, e);
    ascl = 1.f / bl;  // applied after asc: z̄_lap 2^e 2^-eh, each factor within fp32's range
    asct = 1.f / bt;
    bscl = bl;
    bsct = bt;
    osc = ldexpf(1.f, -e);
  }

  floatx4 dacc[RT][NT];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) dacc[i][ct] = floatx4{0.f, 0.f, 0.f, 0.f};

  // raw operands of one chunk, per thread: 4 granules (unit ul = it >> 1, row tile
  // wave + 8 (it & 1)) of z̄_j, z_{j-1} (stream 0) and z_{j-1} (stream s).  The next chunk's
  // loads are issued before the MFMA phase of the current one (software pipeline).
  floatx4 rzb[G], rz0[G], rzs[G];
  // branch-free: a granule past the end loads unit 0 (valid memory) and is zeroed in put(),
  // so the compiler keeps every load of the chunk in flight (no waitcnt inside fetch)
  auto fetch = [&](int ch) {
#pragma unroll
    for (int it = 0; it < G; ++it) {
      const int ul = it / RT, rt = wave + 8 * (it % RT);
      const int u = 2 * ch + ul;
      const int uu = (ch < c1 && u < units) ? u : 0;
      const int t = uu / S, s = uu - t * S;
      const float* ba = abase(t);
      rzb[it] = *reinterpret_cast<const floatx4*>(act_base(adj, j - 1, ntiles, t, S, NT) +
                                                  ((s * NT + rt) * 64 + lane) * 4);
      if (S % 2 != 0 || it < RT) rz0[it] = *reinterpret_cast<const floatx4*>(ba + (rt * 64 + lane) * 4);
      rzs[it] = load_zs<NT, S, LAP>(ba, s, rt, lane, l0, w0, din);
    }
  };
  floatx4 ssv[G], scv[G];
  auto put = [&](int ch) {
#pragma unroll
    for (int it = 0; it < G; ++it) {
      const int ul = it / RT, rt = wave + 8 * (it % RT);
      const int u = 2 * ch + ul;
      const bool live = u < units;
      const int uu = live ? u : 0;
      const int t = uu / S, s = uu - t * S;
      // even S: units 2ch, 2ch + 1 are streams of ONE tile, so granules it and it + RT share z0
      constexpr bool kShare = S % 2 == 0;
      if (!kShare || it < RT) {
        float amax = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) amax = fmaxf(amax, fabsf(OMEGA * rz0[it][r]));
        const bool big = wave_any_big(amax);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float a, b;
          if (big)
            sincosf(OMEGA * rz0[it][r], &a, &b);
          else
            sincos_fast(OMEGA * rz0[it][r], a, b);
          ssv[kShare ? it % RT : it][r] = a;
          scv[kShare ? it % RT : it][r] = b;
        }
      }
      const floatx4 sv = ssv[kShare ? it % RT : it], cv = scv[kShare ? it % RT : it];
      floatx4 hv;
      if (LAP && s == S - 1) {  // Laplacian stream: h = w c q - w^2 s sum_i t_i^2
        if constexpr (S % 2 == 0) {
          // even S: this chunk's first unit is stream S - 2 of the same tile (its z is in
          // registers), and q is this granule's own load -- only tangents 1 .. S - 3 are read
          // (summed in stream order 1 .. S - 2, as h_stream and the forward do)
          const floatx4 zsib = rzs[it >= RT ? it - RT : 0];
          floatx4 t2 = floatx4{0.f, 0.f, 0.f, 0.f};
          const float* ba = abase(t);
#pragma unroll
          for (int ti = 1; ti < S - 2; ++ti) {
            const floatx4 z = load_zs<NT, S, LAP>(ba, ti, rt, lane, l0, w0, din);
#pragma unroll
            for (int r = 0; r < 4; ++r) t2[r] = fmaf(z[r], z[r], t2[r]);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) t2[r] = fmaf(zsib[r], zsib[r], t2[r]);
#pragma unroll
          for (int r = 0; r < 4; ++r) hv[r] = OMEGA * cv[r] * rzs[it][r] - OMEGA2 * sv[r] * t2[r];
        } else {
          hv = h_stream<NT, S, LAP>(abase(t), s, rt, lane, sv, cv, l0, w0, din);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) hv[r] = s == 0 ? sv[r] : OMEGA * cv[r] * rzs[it][r];
      }
      const floatx4 zero = floatx4{0.f, 0.f, 0.f, 0.f};
      if constexpr (NQ == 4) {
        const bool lq = LAP && s == S - 1;
        const float fa = lq ? ascl : (s > 0 ? asct : 1.f), fb = lq ? bscl : (s > 0 ? bsct : 1.f);
        dw_put<NQ, NT>(A, live ? (rzb[it] * asc) * fa : zero, rt, ul, lane);
        dw_put<NQ, NT>(B, live ? hv * fb : zero, rt, ul, lane);
      } else {
        dw_put<NQ, NT>(A, live ? rzb[it] : zero, rt, ul, lane);
        dw_put<NQ, NT>(B, live ? hv : zero, rt, ul, lane);
      }
    }
  };

  fetch(c0);
  for (int ch = c0; ch < c1; ++ch) {
    __syncthreads();  // the previous chunk's MFMA readers are done
    put(ch);
    fetch(ch + 1);
    __syncthreads();
    FragQ<NQ> af[RT];
#pragma unroll
    for (int i = 0; i < RT; ++i) af[i] = lds_frag<NQ, kDwPL>(A + (16 * (RT * wave + i) + c) * kDwKR + 8 * g);
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) {
      const FragQ<NQ> bf = lds_frag<NQ, kDwPL>(B + (16 * ct + c) * kDwKR + 8 * g);
#pragma unroll
      for (int i = 0; i < RT; ++i) dacc[i][ct] = mfma_q<NQ>(af[i], bf, dacc[i][ct]);
    }
  }
  float* out = dpart + ((long)(j - 1) * KS + blockIdx.x) * W * W;
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(16 * (RT * wave + i) + 4 * g + r) * W + 16 * ct + c] = dacc[i][ct][r] * osc;
}

// ---------------------------------------------------------------------------------------
// reductions of the wide path (fixed order, no atomics)
// ---------------------------------------------------------------------------------------
namespace {  // one copy per precision translation unit

// compact rows -> the net's flat gradient (column i of the compact row -> its flat index)
__global__ __launch_bounds__(256) void reduce_small_kernel(const float* __restrict__ part, int nb, long count,
                                                           int din, int dout, int L, int W, float* __restrict__ grad,
                                                           int accumulate) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long i = (long)blockIdx.x * 64 + lane;
  float acc = 0.f;
  if (i < count)
    for (int b = w; b < nb; b += 4) acc += part[(long)b * count + i];
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && i < count) {
    const float t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    const long head = (long)W * din + W, hid = (long)L * W;
    long dst;
    if (i < head)
      dst = i;
    else if (i < head + hid)
      dst = hidden_off(din, W, 1 + (int)((i - head) / W)) + (long)W * W + (i - head) % W;
    else
      dst = out_off(din, W, L) + (i - head - hid);
    grad[dst] = accumulate ? grad[dst] + t : t;
  }
}

// first level of the compact-row reduction: RS row slices -> RS rows (fixed order)
constexpr int kSmallRS = 32;
__global__ __launch_bounds__(256) void reduce_rows_kernel(const float* __restrict__ part, int nb, long count,
                                                          float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long i = (long)blockIdx.x * 64 + lane;
  const int b0 = (int)((long)nb * blockIdx.y / gridDim.y), b1 = (int)((long)nb * (blockIdx.y + 1) / gridDim.y);
  float acc = 0.f;
  if (i < count) {
    int b = b0 + w;
    for (; b + 28 < b1; b += 32) {  // 8 independent loads in flight per thread (fixed order)
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long)(b + 4 * u) * count + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; b < b1; b += 4) acc += part[(long)b * count + i];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && i < count) out[(long)blockIdx.y * count + i] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

// per hidden layer (blockIdx.y < L): sum of the KS partial W x W blocks.  A block = 64 column
// quads (16-B loads, 1 KiB per wave-instruction) x 8 waves over the slices, 8 independent loads
// in flight per thread; fixed summation order (deterministic, no atomics).  Plane y == L: the
// second level of the compact-row reduction (rs rows -> the flat gradient), same launch.
// frag = 1: the partials are in matrix-core fragment order (jet_x6r.hpp: float4 q = (row tile x W / 16 +
// column tile) x 64 + lane holds rows 16 rt + 4 (lane >> 4) + r of column 16 ct + (lane & 15)), so the
// producer's stores are whole 1 KiB wave writes; the sums are scattered to row-major .grad here.
// kstep / kslots: partial k of layer j sits at slot k kstep of the layer's kslots (pair sums: 2, nb)
__global__ __launch_bounds__(512) void reduce_dw_kernel(const float* __restrict__ dpart, int KS, int din, int W,
                                                        float* __restrict__ grad, int accumulate, int grad16, int frag, int L,
                                                        const float* __restrict__ rows, int rs, long Ps, int dout,
                                                        int kstep, int kslots, AdamArgs A) {
  __shared__ floatx4 red[8][64];
  __shared__ float sc[2];  // A.m != NULL: Adam's step size and sqrt(1 - b2^t)
  // A.fin.nloss > 0: block (last column, plane L) -- the grid's extra column, no work of its own --
  // finishes the seeded backward's loss values before its plateau ticket
  if (A.fin.nloss && (int)blockIdx.y == L && blockIdx.x == gridDim.x - 1 && threadIdx.x < 64) loss_finalize(A.fin);
  if (A.m && threadIdx.x == 0) {
    const double t = (double)A.st[INSR_OPT_STEP] + 1.0;
    double p1, p2;
    powi2_d((double)A.b1, (double)A.b2, (unsigned)t, p1, p2);
    sc[0] = (float)((double)A.st[INSR_OPT_LR] / (1.0 - p1));
    sc[1] = (float)sqrt(1.0 - p2);
  }
  // the gradient element grad[i] = g, then (A.m) its Adam update from the state (m0, v0, p0) the thread
  // loaded before the sums -- torch's op order (optim.hpp)
  auto put = [&](long i, float g, float m0, float v0, float p0) {
    grad[i] = g;
    if (A.m) {
      float mi, vi;
      const float pn = adam_elem(g, m0, v0, p0, sc[0], sc[1], (float)(1.0 - (double)A.b1),
                                 (float)(1.0 - (double)A.b2), A.b2, A.eps, mi, vi);
      A.m[i] = mi;
      A.v[i] = vi;
      A.p[i] = pn;
      if (A.shape[2] > 0) adam_wsplit(A.p, A.shape, i, pn);
    }
  };
  float g0 = 0.f, m0 = 0.f, v0 = 0.f, p0 = 0.f;  // this thread's element's state (its epilogue)
  auto preload = [&](long i) {
    if (accumulate) g0 = grad[i];
    if (A.m) {
      m0 = A.m[i];
      v0 = A.v[i];
      p0 = A.p[i];
    }
  };
  if ((int)blockIdx.y == L) {
    float* r = reinterpret_cast<float*>(&red[0][0]);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long i = (long)blockIdx.x * 64 + lane;
    const long head = (long)W * din + W, hid = (long)L * W;
    long dst = 0;
    if (i < Ps) {
      if (i < head)
        dst = i;
      else if (i < head + hid)
        dst = hidden_off(din, W, 1 + (int)((i - head) / W)) + (long)W * W + (i - head) % W;
      else
        dst = out_off(din, W, L) + (i - head - hid);
      if (w == 0) preload(dst);
    }
    float acc = 0.f;
    if (i < Ps) {  // 16 rows in flight per thread, as the W x W planes (a fixed order all the same)
      for (int b = w; b < rs; b += 128) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = b + 8 * u < rs ? rows[(long)(b + 8 * u) * Ps + i] : 0.f;
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += v[u];
      }
    }
    r[w * 64 + lane] = acc;
    __syncthreads();
    if (w == 0 && i < Ps) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) t += r[k * 64 + lane];
      put(dst, accumulate ? g0 + t : t, m0, v0, p0);
    }
  } else {
    const int j = blockIdx.y + 1;
    const long WW = (long)W * W;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long q = (long)blockIdx.x * 64 + lane;  // column quad
    // frag = 1: the quad's 4 elements are rows 16 (f / nt) + 4 (ln >> 4) + r of one column; wave r < 4
    // runs element r's epilogue (its state loaded here, under the sums)
    const int ln = (int)(q & 63), f = (int)(q >> 6), nt = W / 16;
    const long d0 = hidden_off(din, W, j) + (long)(16 * (f / nt) + 4 * (ln >> 4)) * W + 16 * (f % nt) + (ln & 15);
    // frag = 0 (row-major partials) with an Adam epilogue: the quad's 4 consecutive elements alike
    const bool per_elem = frag || A.m;
    auto elem = [&](int r) -> long { return frag ? d0 + (long)r * W : hidden_off(din, W, j) + 4 * q + r; };
    if (per_elem && w < 4 && 4 * q < WW) preload(elem(w));
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
    if (4 * q < WW) {
      const floatx4* col = reinterpret_cast<const floatx4*>(dpart + (long)(j - 1) * kslots * WW) + q;
      const long rs4 = WW / 4 * kstep;
      // slices w, w + 8, ... in order, 16 in flight per thread (a batch's slices past KS add zeros)
      for (int k = w; k < KS; k += 128) {
        floatx4 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = k + 8 * u < KS ? col[(long)(k + 8 * u) * rs4] : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += v[u];
      }
    }
    red[w][lane] = acc;
    __syncthreads();
    if (per_elem) {
      if (w == 0 && 4 * q < WW) {  // the cross-wave sums in the fixed order, back into red[0]
        floatx4 t = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 8; ++k) t += red[k][lane];
        red[0][lane] = t;
      }
      __syncthreads();
      if (w < 4 && 4 * q < WW) {
        const float t = red[0][lane][w];
        put(elem(w), accumulate ? g0 + t : t, m0, v0, p0);
      }
    } else if (w == 0 && 4 * q < WW) {  // row-major partials, no epilogue: one 16-B store per quad
      floatx4 t = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 8; ++k) t += red[k][lane];
      {
        float* dst = grad + hidden_off(din, W, j) + 4 * q;
        if (grad16) {  // the gradient buffer's hidden blocks are 16-B aligned (a net's own flat .grad)
          floatx4* d4 = reinterpret_cast<floatx4*>(dst);
          if (accumulate) t += *d4;
          *d4 = t;
        } else {  // e.g. a slice of a data-parallel gradient arena
#pragma unroll
          for (int r = 0; r < 4; ++r) dst[r] = accumulate ? dst[r] + t[r] : t[r];
        }
      }
    }
  }
  if (A.m && A.loss) plateau_after_blocks(A.st, A.loss, A.patience, blockIdx.y * gridDim.x + blockIdx.x,
                                          gridDim.x * gridDim.y);
}

}  // namespace

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
inline int wide_ks(long n, int S, int L) {
  const long chunks = (((n + 15) / 16) * S + 1) / 2;
  long ks = 512 / (L > 0 ? L : 1);  // L x KS <= 512 blocks: two full rounds of 256 one-block CUs
  if (ks > chunks) ks = chunks;
  return ks < 1 ? 1 : (int)ks;
}

// workspace floats: z̄ of the L hidden layers | compact rows | dW partials | rows
inline long wide_work_floats_impl(long n, int din, int dout, int L, int W, int S) {
  const long ntiles = ((n + 63) / 64) * 4;
  const long adj = (long)L * ntiles * S * (W / 16) * 256;
  const long small = ((n + 15) / 16) * small_count(din, dout, L, W);
  const long dw = (long)L * wide_ks(n, S, L) * W * W;
  const long zmax = 19L * L * ((n + 15) / 16);  // tile maxima of the adjoints and h bounds (fp16 dW)
  return adj + small + dw + (long)kSmallRS * small_count(din, dout, L, W) + zmax;
}

// threads of the three launches of wide_bwd_t (L > 0): propagation, dW + rows level 1,
// dW sums + rows level 2 (the launch shapes rocprof reports; bench.py's traffic lookup)
inline void wide_launch_threads_impl(long n, int din, int dout, int L, int W, int S, long* out) {
  const long tiles = (n + 15) / 16, Ps = small_count(din, dout, L, W);
  const long rs = tiles < kSmallRS ? tiles : kSmallRS, rows_x = (Ps + 63) / 64;
  const long KS = wide_ks(n, S, L), planes = (rows_x * rs + KS - 1) / KS;
  const long wq = ((long)W * W / 4 + 63) / 64;
  out[0] = tiles * 512;
  out[1] = KS * (L + planes) * 512;
  out[2] = (wq > rows_x ? wq : rows_x) * (L + 1) * 512;
}

// phases (L > 0): 1 the propagation + dW partials, 2 the sums (with A.m: + the Adam update), 3 both
template <int NQ, int NT, int S, bool LAP>
// J: the jobs (one for a single call); N: the layout count, 16 x the jobs' tiles for several (a single
// call passes its own n) -- the workspace, KS and the sums launch all follow N, so a phase-2 call with the
// same N finds what phase 1 wrote
int wide_bwd_t(const FbJobs& J, int N, int din, int dout, int L, const float* prm, float* work, float* grad,
               int accumulate, int f16, int phases, const AdamArgs& A, hipStream_t st) {
  constexpr int W = 16 * NT;
  const long ntiles = ((N + 63) / 64) * 4;
  const int tiles = (N + 15) / 16;
  const long Ps = small_count(din, dout, L, W);
  float* adj = work;
  float* small = adj + (long)L * ntiles * S * NT * 256;
  float* dpart = small + (long)tiles * Ps;
  float* rows = dpart + (long)L * wide_ks(N, S, L) * W * W;
  float* zmax = rows + (long)kSmallRS * Ps;
  // the x6 precision's products on the fp16 matrix cores (dw_x6 / jet_bwd_x6p NQ = 4, above)
  const bool f16dw = NQ == 3 && (f16 & INSR_BWD_F16_DW) && L > 0;
  const bool f16p = NQ == 3 && (f16 & INSR_BWD_F16_PROP) && L > 0;
  constexpr size_t lds_p = (size_t)S * np_of<NQ>() * 16 * (W + 8) * 2 + 2 * 3 * 8 * sizeof(float);
  constexpr size_t lds_p4 = (size_t)S * 2 * 16 * (W + 8) * 2 + 2 * 3 * 8 * sizeof(float);
  static const bool attr = [] {  // once per instantiation (thread-safe static init)
    (void)hipFuncSetAttribute((const void*)jet_bwd_x6p<NQ, NT, S, LAP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds_p);
    (void)hipFuncSetAttribute((const void*)dw_x6<NQ, NT, S, LAP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)dw_lds<NQ, NT>());
    if constexpr (NQ == 3) {
      (void)hipFuncSetAttribute((const void*)dw_x6<4, NT, S, LAP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)dw_lds<4, NT>());
      (void)hipFuncSetAttribute((const void*)jet_bwd_x6p<4, NT, S, LAP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds_p4);
    }
    return true;
  }();
  (void)attr;
  if (L == 0 && phases != 3) return INSR_EINVAL;  // (the phase split is for the hidden-layer sums)
  const int rs = tiles < kSmallRS ? tiles : kSmallRS;
  const int rows_x = (int)((Ps + 63) / 64);
  if (!(phases & 1)) {  // the sums alone
    const int KS = wide_ks(N, S, L);
    const int grad16 = (((uintptr_t)(grad + hidden_off(din, W, 1))) & 15) == 0 ? 1 : 0;
    const int wq = (W * W / 4 + 63) / 64;
    hipLaunchKernelGGL(reduce_dw_kernel, dim3((unsigned)(wq > rows_x ? wq : rows_x), L + 1), dim3(512), 0, st, dpart,
                       KS, din, W, grad, accumulate, grad16, 0, L, rows, rs, Ps, dout, 1, KS, A);
    return (int)hipGetLastError();
  }
  bool launched = false;
  if constexpr (NQ == 3) {
    if (f16p) {
      hipLaunchKernelGGL((jet_bwd_x6p<4, NT, S, LAP>), dim3(tiles), dim3(512), lds_p4, st, J, N, din, dout, L, prm, adj,
                         small, Ps, f16dw ? zmax : nullptr);
      launched = true;
    }
  }
  if (!launched)
    hipLaunchKernelGGL((jet_bwd_x6p<NQ, NT, S, LAP>), dim3(tiles), dim3(512), lds_p, st, J, N, din, dout, L, prm, adj,
                       small, Ps, f16dw ? zmax : nullptr);
  if (L > 0) {  // 3 launches: propagation | dW partials + compact rows level 1 | dW sums + rows level 2
    const int KS = wide_ks(N, S, L);
    const int planes = (rows_x * rs + KS - 1) / KS;
    bool done = false;
    if constexpr (NQ == 3) {
      if (f16dw) {
        hipLaunchKernelGGL((dw_x6<4, NT, S, LAP>), dim3(KS, L + planes), dim3(512), (dw_lds<4, NT>()), st, N, J, adj,
                           dpart, KS, L, small, tiles, Ps, rows, rs, rows_x, zmax, prm, din);
        done = true;
      }
    }
    if (!done)
      hipLaunchKernelGGL((dw_x6<NQ, NT, S, LAP>), dim3(KS, L + planes), dim3(512), (dw_lds<NQ, NT>()), st, N, J, adj,
                         dpart, KS, L, small, tiles, Ps, rows, rs, rows_x, zmax, prm, din);
    if (!(phases & 2)) return (int)hipGetLastError();
    const int grad16 = (((uintptr_t)(grad + hidden_off(din, W, 1))) & 15) == 0 ? 1 : 0;  // W % 4 == 0: all layers alike
    const int wq = (W * W / 4 + 63) / 64;
    hipLaunchKernelGGL(reduce_dw_kernel, dim3((unsigned)(wq > rows_x ? wq : rows_x), L + 1), dim3(512), 0, st, dpart,
                       KS, din, W, grad, accumulate, grad16, 0, L, rows, rs, Ps, dout, 1, KS, A);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(reduce_rows_kernel, dim3((unsigned)rows_x, rs), dim3(256), 0, st, small, tiles, Ps, rows);
  hipLaunchKernelGGL(reduce_small_kernel, dim3((unsigned)rows_x), dim3(256), 0, st, rows, rs, Ps, din, dout, L, W, grad,
                     accumulate);
  return (int)hipGetLastError();
}

template <int NQ, int NT>
int wide_bwd_nt(int S, bool LAP, const FbJobs& J, int N, int din, int dout, int L, const float* prm, float* work,
                float* grad, int accumulate, int f16, int phases, const AdamArgs& A, hipStream_t st) {
  switch (S * 2 + (LAP ? 1 : 0)) {
    case 2: return wide_bwd_t<NQ, NT, 1, false>(J, N, din, dout, L, prm, work, grad, accumulate, f16, phases, A, st);
    case 4: return wide_bwd_t<NQ, NT, 2, false>(J, N, din, dout, L, prm, work, grad, accumulate, f16, phases, A, st);
    case 6: return wide_bwd_t<NQ, NT, 3, false>(J, N, din, dout, L, prm, work, grad, accumulate, f16, phases, A, st);
    case 8: return wide_bwd_t<NQ, NT, 4, false>(J, N, din, dout, L, prm, work, grad, accumulate, f16, phases, A, st);
    case 7: return wide_bwd_t<NQ, NT, 3, true>(J, N, din, dout, L, prm, work, grad, accumulate, f16, phases, A, st);
    case 9: return wide_bwd_t<NQ, NT, 4, true>(J, N, din, dout, L, prm, work, grad, accumulate, f16, phases, A, st);
    case 11: return wide_bwd_t<NQ, NT, 5, true>(J, N, din, dout, L, prm, work, grad, accumulate, f16, phases, A, st);
    default: return INSR_EINVAL;
  }
}

template <int NQ>
int dispatch_wide_bwd_q(int NT, int S, bool LAP, const FbJobs& J, int N, int din, int dout, int L, const float* prm,
                        float* work, float* grad, int accumulate, int f16, int phases, const AdamArgs& A,
                        hipStream_t st) {
  if (NT == 16)
    return wide_bwd_nt<NQ, 16>(S, LAP, J, N, din, dout, L, prm, work, grad, accumulate, f16, phases, A, st);
  if (NT == 8)
    return wide_bwd_nt<NQ, 8>(S, LAP, J, N, din, dout, L, prm, work, grad, accumulate, f16, phases, A, st);
  return INSR_EWIDTH;
}

}  // namespace insr
#endif  // INSR_WIDE_NQ_DEFS
