// advect_iter.hip -- one launch for the forward, residual and reverse of an advection iteration.
//
// The reference's 1-D advection phase (advection/model.py:68-91) on a 1 -> 1 SIREN of L hidden 64 x 64
// layers: per iteration it draws 4,096 collocation points and a 2 x 20-point Dirichlet band
// (base/sampling.py:14-30), evaluates the frozen field and the trainable one with their x-derivatives
// (diff_ops.gradient, base/diff_ops.py:44-58), forms
//   main = mean(((u - u0) / dt + vel (u_x + u0_x) / 2)^2),  bc = mean(u_band^2)
// and back-propagates into the trainable field.  The generic path spends five latency-bound launches
// on it (sampler, mixed forward, loss group, reverse jet, sums + Adam: ~50 us for a 50 KB network).
// Here ONE launch does everything but the sums: each block (4 waves, wave w owning neuron rows
// 16 w .. 16 w + 15 of every hidden layer) walks its share of the 16-point tiles and per tile
//   draws its points (the Philox-4x32-10 stream of insr_sample_boxes, bit-identical to the three-box
//     draw of the fused model's one sampler launch; the last block advances the device stream),
//   runs both fields' value + tangent jets (layer 0 on the VALU, hidden layers as exact-fp32
//     v_mfma_f32_16x16x4_f32 GEMMs over (streams x 16 points), the two fields interleaved for ILP),
//   forms the residuals and their adjoint seeds (fixed-order cross-wave sums, no loss launch),
//   runs the reverse jet of the trainable field: sine reverse (lane-local), dW_j = Z̄_j H_{j-1}^T on
//     the matrix cores (accumulated in registers over the block's tiles), H̄_{j-1} = W_j^T Z̄_j,
// and writes ONE partial-gradient row; the last block (a ticket) finishes the two loss values from the
// blocks' sums and advances the sampler stream.  insr_adam_step_partials sums the rows with the Adam (+
// plateau) update of every parameter: an iteration is two launches.  Exact fp32 products throughout (the oracle's arithmetic up to the
// summation order).
#include "jet_common.hpp"

namespace insr {

constexpr int kAdvW = 64;        // hidden width (4 row tiles = 4 waves)
constexpr int kAdvThreads = 512;  // 8 waves (two per SIMD)
constexpr int kAdvLD = 68;       // LDS row stride of a point-major [16 points][64 + 4] plane
constexpr int kAdvPlane = 16 * kAdvLD;

// Diagnostic phase stamps (the diag library only, -DINSR_STAMPS; tools/adv_iter_study.py): s_memtime at the
// phase boundaries of block 0's first tile, [wave][stamp]
#ifdef INSR_STAMPS
constexpr int kAdvStamps = 32;
static __device__ unsigned long long g_adv_stamps[8 * kAdvStamps];
#define ADV_STAMP(k)                                                                                       \
  do {                                                                                                     \
    if (blockIdx.x == 0 && lane == 0 && tile == (int)blockIdx.x) g_adv_stamps[wave * kAdvStamps + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define ADV_STAMP(k) \
  do {               \
  } while (0)
#endif

struct AdvectPk {
  const float* prm;   // trainable field, flat (state_dict order)
  const float* prev;  // frozen field
  float* part;        // [nb][stride] partial gradient rows
  float* lpart;       // [nb][INSR_SEED_MAX]: 0 = sum of interior residual^2, 1 = sum of band u^2
  float* xout;        // the drawn points (n + 2h) or NULL
  unsigned long long* state;  // sampler state: Philox counter, ticket
  unsigned long long seed;
  long stride;
  int n, h, tiles, nb;
  float lo[3], hi[3];  // the three boxes: interior, band at -L/2, band at +L/2
  float inv_dt, hvel;  // 1 / dt, vel / 2
  float gmain, gbc;    // 2 / (interior total), 2 / (band total): d mean / d residual = g * r
  float* loss;         // [2]: main, bc (the last block's combine)
  float smain, sbc;    // 1 / (interior total), 1 / (band total)
};

__device__ __forceinline__ uint4 adv_philox(unsigned long long key, unsigned long long ctr) {
  unsigned c0 = (unsigned)ctr, c1 = (unsigned)(ctr >> 32), c2 = 0u, c3 = 0u;
  unsigned k0 = (unsigned)key, k1 = (unsigned)(key >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const unsigned hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const unsigned n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return uint4{c0, c1, c2, c3};
}

// sin / cos of w z for a lane's 4 rows (the ocml path for a wave holding any |w z| > 8192)
__device__ __forceinline__ void adv_sincos(const floatx4& z, floatx4& s, floatx4& c) {
  float amax = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) amax = fmaxf(amax, fabsf(OMEGA * z[r]));
  const bool big = wave_any_big(amax);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float a, b;
    if (big)
      sincosf(OMEGA * z[r], &a, &b);
    else
      sincos_fast(OMEGA * z[r], a, b);
    s[r] = a;
    c[r] = b;
  }
}

// LDS (floats): WS [2 fields][L][W][68] the hidden weights of both fields, staged once per block with
// coalesced 16-B loads (row stride 68); SM [2][193 + 64 L, padded] their W_0, b_0, b_j, W_out, b_out; then
// POINT-major [16 points][68] planes: HT [L][2] the trainable field's h / dh of sine layers 0 .. L-1 (the
// next layer's and dW's B operand), HP [2] the frozen field's (ping-pong with ZB's first buffer during the
// forward), ZB [2][2] the adjoints z̄ / t̄ (double-buffered by layer); RED [2 fields][4][2][16] the output
// layer's per-row-tile sums; SD [2][16] the tile's adjoint seeds.  L = 3: 160,928 bytes (one block per CU).
// Point-major planes and a permuted K order (MFMA step kc, lane group g: k = 16 g + kc) make every GEMM
// operand that walks K a run of 16 consecutive floats in LDS: 4 ds_read_b128 instead of 16 ds_read_b32.
constexpr int kAdvWLD = 68;
template <int L>
constexpr int adv_small() { return (193 + 64 * L + 3) & ~3; }
template <int L>
constexpr int adv_lds_floats() {
  return 2 * L * kAdvW * kAdvWLD + 2 * adv_small<L>() + (L * 2 + 2 + 4) * kAdvPlane + 2 * 4 * 2 * 16 + 2 * 16;
}

__device__ __forceinline__ void lds_get16(const float* p, float (&v)[16]) {
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const floatx4 q = *reinterpret_cast<const floatx4*>(p + 4 * m);
    v[4 * m] = q[0];
    v[4 * m + 1] = q[1];
    v[4 * m + 2] = q[2];
    v[4 * m + 3] = q[3];
  }
}

// Block = 8 waves.  Forward: waves 0-3 run the trainable field, waves 4-7 the frozen one (wave & 3 = the
// row tile: neurons 16 (w & 3) .. + 15 of every hidden layer).  Reverse: waves 0-3 the sine reverse and
// the propagation h̄_{j-1} = W_j^T z̄_j, waves 4-7 dW_j = Z̄_j H_{j-1}^T (register accumulators over the
// block's tiles) -- the two GEMMs of a layer in parallel.
template <int L>
__global__ __launch_bounds__(kAdvThreads) void advect1d_iter_kernel(const AdvectPk pk) {
  constexpr int W = kAdvW, LD = kAdvLD, PL = kAdvPlane, WL = kAdvWLD, SMN = adv_small<L>();
  static_assert(LD * 16 == PL, "point-major planes: [16 points][LD]");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* WS = lds;                      // [q][j - 1][row][68]
  float* SM = WS + 2 * L * W * WL;      // [q][SMN]: W_0 | b_0 | b_1 .. b_L | W_out | b_out
  float* HT = SM + 2 * SMN;
  float* HP = HT + L * 2 * PL;
  float* ZB = HP + 2 * PL;
  float* RED = ZB + 4 * PL;
  float* SD = RED + 2 * 4 * 2 * 16;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int grp = wave >> 2, wg = wave & 3;  // field (forward) / role (reverse), row tile
  const int g = lane >> 4, c = lane & 15;
  const int n0 = 16 * wg + 4 * g;  // this lane's first neuron of every hidden layer
  const unsigned long long base = pk.state[0];
  const int total = pk.n + 2 * pk.h;
  const float* P[2] = {pk.prm, pk.prev};  // 0: trainable, 1: frozen
  const long wout = out_off(1, W, L);
  constexpr int kB = 128, kWo = 128 + 64 * L;  // SM offsets of b_1 and W_out (b_out at kWo + 64)
  const float* SMq = SM + grp * SMN;           // this wave's field's small parameters (forward)

  // ---- stage both fields' parameters (every later weight read is LDS): all of a thread's 16-B loads are
  // issued before its first LDS store (one L2 / HBM latency per block, not one per load) ----
  {
    constexpr int NV = L * W * W / 4 / kAdvThreads;  // float4 per thread and field (L = 3: 6)
    static_assert(NV * kAdvThreads == L * W * W / 4, "staging split");
    floatx4 v[2][NV];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        const int i = tid + u * kAdvThreads;
        const int j = i / (W * W / 4), rem = i - j * (W * W / 4);
        v[q][u] = *reinterpret_cast<const floatx4*>(P[q] + hidden_off(1, W, j + 1) + 4 * rem);
      }
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        const int i = tid + u * kAdvThreads;
        const int j = i / (W * W / 4), rem = i - j * (W * W / 4), row = rem >> 4, c4 = rem & 15;
        *reinterpret_cast<floatx4*>(WS + ((q * L + j) * W + row) * WL + 4 * c4) = v[q][u];
      }
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    for (int k = tid; k < 193 + 64 * L; k += kAdvThreads) {
      long src;
      if (k < kB)
        src = k;
      else if (k < kWo)
        src = hidden_off(1, W, 1 + (k - kB) / W) + (long)W * W + (k - kB) % W;
      else
        src = wout + (k - kWo);
      SM[q * SMN + k] = P[q][src];
    }
  }

  floatx4 dacc[L][4];  // waves 4-7: dW_j rows of this row tile x column tile ct, over the block's tiles
#pragma unroll
  for (int j = 0; j < L; ++j)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) dacc[j][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
  // waves 0-3: compact sums of this lane's rows n0 .. n0 + 3 (every lane of a 16-lane row holds the sums)
  floatx4 gW0 = {0.f, 0.f, 0.f, 0.f}, gb0 = {0.f, 0.f, 0.f, 0.f}, gWo = {0.f, 0.f, 0.f, 0.f};
  floatx4 gb[L];
#pragma unroll
  for (int j = 0; j < L; ++j) gb[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float gbo = 0.f, lmain = 0.f, lbc = 0.f;

  // tiles b, b + nb, b + 2 nb, ... (nb = min(tiles, CUs)): the advect1D batch's 256 interior tiles one per
  // block, its 3 band tiles the second tile of blocks 0-2.  A band tile (every point a band point) needs
  // neither the frozen field (no residual) nor the tangent streams (u_x enters no band term: their
  // adjoints are zero), so its frozen waves skip the forward and every tangent product is skipped --
  // the critical path is one interior tile plus that lighter one instead of two interior tiles.
  for (int tile = blockIdx.x; tile < pk.tiles; tile += pk.nb) {
    const bool band = tile * 16 >= pk.n;  // (uniform)
    const bool work = !(band && grp == 1);  // this wave's forward runs
    __syncthreads();  // the staged parameters / the previous tile's last readers of HT, ZB, RED, SD
    ADV_STAMP(0);
    // ---- the tile's points: value v of the draw = lo + (hi - lo) u(v), u from Philox(seed, base + v / 4)
    const int p = tile * 16 + c;
    const bool valid = p < total;
    float x = 0.f;
    if (valid) {
      const uint4 r4 = adv_philox(pk.seed, base + (unsigned long long)(p >> 2));
      const unsigned bits = (p & 3) == 0 ? r4.x : (p & 3) == 1 ? r4.y : (p & 3) == 2 ? r4.z : r4.w;
      const int k = p < pk.n ? 0 : (p < pk.n + pk.h ? 1 : 2);
      const float u = (float)(bits >> 8) * 5.9604644775390625e-8f;  // 2^-24 (sampler.hip)
      const float lo = pk.lo[k], hi = pk.hi[k];
      x = lo + (hi - lo) * u;
      if (pk.xout && g == 0 && wave == 0) pk.xout[p] = x;
    }

    // ---- forward: this wave's field, value (stream 0) and tangent (stream 1) ----
    floatx4 zs[L + 1], ts[L + 1];  // z / t of sine layers 0 .. L (the trainable field's: the reverse's)
    if (work) {
      floatx4 z, t, s, cs;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float w0 = SMq[n0 + r];
        z[r] = fmaf(w0, x, SMq[W + n0 + r]);
        t[r] = w0;
      }
      zs[0] = z;
      ts[0] = t;
      adv_sincos(z, s, cs);
      float* H = grp == 0 ? HT : HP;  // layer 0: HT slot 0 / HP
      *reinterpret_cast<floatx4*>(H + c * LD + n0) = s;
      *reinterpret_cast<floatx4*>(H + PL + c * LD + n0) = OMEGA * cs * t;
    }
    ADV_STAMP(1);
    __syncthreads();
#pragma unroll
    for (int j = 1; j <= L; ++j) {
      // B = h_{j-1}[16 g + kc][point c] (point-major: 16 consecutive floats), A = W_j[16 wg + c][16 g + kc]
      floatx4 av = {0.f, 0.f, 0.f, 0.f}, at = {0.f, 0.f, 0.f, 0.f};
      if (work) {
        const float* Bq = grp == 0 ? HT + (j - 1) * 2 * PL : (((j - 1) & 1) ? ZB : HP);
        float a[16], bv[16];
        lds_get16(WS + ((grp * L + j - 1) * W + 16 * wg + c) * WL + 16 * g, a);
        lds_get16(Bq + c * LD + 16 * g, bv);
#pragma unroll
        for (int r = 0; r < 4; ++r) av[r] = SMq[kB + 64 * (j - 1) + n0 + r];
        if (band) {  // value stream only
#pragma unroll
          for (int kc = 0; kc < 16; ++kc) av = mfma4(a[kc], bv[kc], av);
        } else {
          float bt[16];
          lds_get16(Bq + PL + c * LD + 16 * g, bt);
#pragma unroll
          for (int kc = 0; kc < 16; ++kc) {
            av = mfma4(a[kc], bv[kc], av);
            at = mfma4(a[kc], bt[kc], at);
          }
        }
      }
      zs[j] = av;
      ts[j] = at;
      if (j < L) {  // h_j -> LDS (the next layer's B operand; the trainable one also dW's)
        if (work) {
          floatx4 s, cs;
          adv_sincos(av, s, cs);
          float* Hn = grp == 0 ? HT + j * 2 * PL : ((j & 1) ? ZB : HP);
          *reinterpret_cast<floatx4*>(Hn + c * LD + n0) = s;
          *reinterpret_cast<floatx4*>(Hn + PL + c * LD + n0) = OMEGA * cs * at;  // (band: zeros)
        }
        __syncthreads();
      }
    }
    ADV_STAMP(2);
    // output layer (exact fp32 VALU): y = W_out h_L + b_out, y_x = W_out dh_L of this wave's field: its
    // rows, then the 16-lane rows (g), then the row tiles in a fixed order
    floatx4 sL, cL;
    adv_sincos(zs[L], sL, cL);
    {
      float acc0 = 0.f, acc1 = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float wt = work ? SMq[kWo + n0 + r] : 0.f;  // (a band tile's frozen waves: zeros)
        acc0 = fmaf(wt, sL[r], acc0);
        acc1 = fmaf(wt, OMEGA * cL[r] * ts[L][r], acc1);
      }
      acc0 += __shfl_xor(acc0, 16);
      acc0 += __shfl_xor(acc0, 32);
      acc1 += __shfl_xor(acc1, 16);
      acc1 += __shfl_xor(acc1, 32);
      if (g == 0) {
        RED[((grp * 4 + wg) * 2) * 16 + c] = acc0;
        RED[((grp * 4 + wg) * 2 + 1) * 16 + c] = acc1;
      }
    }
    __syncthreads();
    if (wave == 0 && lane < 16) {  // residuals, seeds and loss sums of the tile's points
      float y[4];
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const float* rq = RED + (q * 4 * 2 + k) * 16 + c;
          y[2 * q + k] = ((rq[0] + rq[2 * 16]) + rq[4 * 16]) + rq[6 * 16];
        }
      const float u = y[0] + SM[kWo + W], ux = y[1], u0 = y[2] + SM[SMN + kWo + W], u0x = y[3];
      float gy = 0.f, gdy = 0.f;
      if (valid && p < pk.n) {
        const float res = (u - u0) * pk.inv_dt + pk.hvel * (ux + u0x);
        lmain = fmaf(res, res, lmain);
        gy = pk.gmain * res * pk.inv_dt;
        gdy = pk.gmain * res * pk.hvel;
      } else if (valid) {
        lbc = fmaf(u, u, lbc);
        gy = pk.gbc * u;
      }
      SD[c] = gy;
      SD[16 + c] = gdy;
    }
    __syncthreads();
    ADV_STAMP(3);

    // ---- reverse (the trainable field): waves 0-3 sine reverse + propagation, waves 4-7 dW ----
    const float gy = SD[c], gdy = SD[16 + c];
    floatx4 hv, ht;  // adjoints of h_j / dh_j
    if (grp == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float wo = SM[kWo + n0 + r];
        hv[r] = wo * gy;
        ht[r] = wo * gdy;
        gWo[r] += sum16(fmaf(gy, sL[r], gdy * (OMEGA * cL[r] * ts[L][r])));
      }
      if (wave == 0) gbo += sum16(g == 0 ? gy : 0.f);
    }
    floatx4 s = sL, cs = cL;
#pragma unroll
    for (int j = L; j >= 1; --j) {
      float* Z = ZB + (j & 1) * 2 * PL;
      if (grp == 0) {  // sine reverse: z̄ = w c h̄ - w^2 s t dh̄, t̄ = w c dh̄ -> Z (point-major)
        floatx4 zb, tb;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          zb[r] = OMEGA * cs[r] * hv[r] - OMEGA2 * s[r] * ts[j][r] * ht[r];
          tb[r] = OMEGA * cs[r] * ht[r];
          gb[j - 1][r] += sum16(zb[r]);
        }
        *reinterpret_cast<floatx4*>(Z + c * LD + n0) = zb;
        *reinterpret_cast<floatx4*>(Z + PL + c * LD + n0) = tb;
      }
      __syncthreads();
      if (grp == 0) {
        // propagation: h̄_{j-1} = W_j^T z̄, dh̄_{j-1} = W_j^T t̄: A = W_j[16 g + kc][16 wg + c], B = z̄[16 g + kc][c]
        const float* AT = WS + ((j - 1) * W + 16 * g) * WL + 16 * wg + c;
        float bv[16], bt[16];
        lds_get16(Z + c * LD + 16 * g, bv);
        lds_get16(Z + PL + c * LD + 16 * g, bt);
        floatx4 nv = {0.f, 0.f, 0.f, 0.f}, nt = {0.f, 0.f, 0.f, 0.f};
        if (band) {  // zero tangent adjoints: the value stream only
#pragma unroll
          for (int kc = 0; kc < 16; ++kc) nv = mfma4(AT[kc * WL], bv[kc], nv);
        } else {
#pragma unroll
          for (int kc = 0; kc < 16; ++kc) {
            const float a = AT[kc * WL];
            nv = mfma4(a, bv[kc], nv);
            nt = mfma4(a, bt[kc], nt);
          }
        }
        hv = nv;
        ht = nt;
        adv_sincos(zs[j - 1], s, cs);
      } else {
        // dW_j rows 16 wg .. x all columns: K = (stream, point) 32 deep in the order k = 8 g + kk (stream
        // k >> 4, point k & 15); A = z̄[n = 16 wg + c] at that (stream, point), B = h_{j-1}[16 ct + c] there
        const float* Hj = HT + (j - 1) * 2 * PL;
        const int st = g >> 1, pb = 8 * (g & 1);
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const float* zr = Z + st * PL + (pb + kk) * LD;
          const float* hr = Hj + st * PL + (pb + kk) * LD;
          const float a = zr[16 * wg + c];
#pragma unroll
          for (int ct = 0; ct < 4; ++ct) dacc[j - 1][ct] = mfma4(a, hr[16 * ct + c], dacc[j - 1][ct]);
        }
      }
    }
    if (grp == 0) {  // first layer (exact fp32 VALU): z_0 = W_0 x + b_0, t_0 = W_0
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float zb = OMEGA * cs[r] * hv[r] - OMEGA2 * s[r] * ts[0][r] * ht[r];
        const float tb = OMEGA * cs[r] * ht[r];
        gb0[r] += sum16(zb);
        gW0[r] += sum16(fmaf(zb, x, tb));
      }
    }
    ADV_STAMP(31);
  }

  // ---- the block's partial row (flat parameter order) and its loss sums ----
  float* row = pk.part + (long)blockIdx.x * pk.stride;
  if (grp == 1) {
#pragma unroll
    for (int j = 0; j < L; ++j) {
      float* dW = row + hidden_off(1, W, j + 1);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) dW[(long)(n0 + r) * W + 16 * ct + c] = dacc[j][ct][r];
    }
  }
  if (grp == 0 && c == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      row[n0 + r] = gW0[r];
      row[W + n0 + r] = gb0[r];
      row[wout + n0 + r] = gWo[r];
#pragma unroll
      for (int j = 0; j < L; ++j) row[hidden_off(1, W, j + 1) + (long)W * W + n0 + r] = gb[j][r];
    }
  }
  if (wave == 0 && lane == 0) row[wout + W] = gbo;
  if (wave == 0) {  // the tile sums of lanes 0 .. 15 (fixed order), as sc1 stores (residual.hip hand-off)
    float a = lmain, b = lbc;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
      a += __shfl_xor(a, off);
      b += __shfl_xor(b, off);
    }
    if (lane == 0) {
      float* lp = pk.lpart + (long)blockIdx.x * INSR_SEED_MAX;
      __hip_atomic_store(lp, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(lp + 1, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // one ticket per block: the last one advances the sampler stream (every block has read `base` by then)
  // and finishes the two loss values from the blocks' sums (fixed order) -- the plateau step of the sums
  // launch and the host read them like any loss
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's sc1 stores are acknowledged
    unsigned* ticket = reinterpret_cast<unsigned*>(pk.state + 1);
    last = atomicAdd(ticket, 1u) == gridDim.x - 1 ? 1 : 0;
    if (last) pk.state[0] = base + (unsigned long long)((total + 3) / 4);
  }
  __syncthreads();
  if (last && wave == 0) {
    float a = 0.f, b = 0.f;
    for (int q = lane; q < (int)gridDim.x; q += 64) {
      a += __hip_atomic_load(pk.lpart + (long)q * INSR_SEED_MAX, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      b += __hip_atomic_load(pk.lpart + (long)q * INSR_SEED_MAX + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      a += __shfl_xor(a, off);
      b += __shfl_xor(b, off);
    }
    if (lane == 0) {
      pk.loss[0] = a * pk.smain;
      pk.loss[1] = b * pk.sbc;
      atomicExch(reinterpret_cast<unsigned*>(pk.state + 1), 0u);
    }
  }
}

// blocks: one per tile up to one per CU (one block per CU: its staged weights fill the LDS); the tiles past
// that are dealt round-robin (advect1d_iter_kernel) -- the 4,136-point advect1D batch is 259 tiles: 256
// blocks, blocks 0-2 also take the three band tiles
inline int adv_blocks(long tiles) {
  const long cus = device_cus();
  return (int)(tiles < 1 ? 1 : (tiles < cus ? tiles : cus));
}

template <int L>
int advect_launch(AdvectPk& pk, hipStream_t st) {
  constexpr size_t lds = (size_t)adv_lds_floats<L>() * sizeof(float);
  static_assert(lds <= 163840, "LDS");
  static const bool attr = ((void)hipFuncSetAttribute((const void*)advect1d_iter_kernel<L>,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                            true);  // once per instantiation (thread-safe static init)
  (void)attr;
  hipLaunchKernelGGL((advect1d_iter_kernel<L>), dim3(pk.nb), dim3(kAdvThreads), lds, st, pk);
  return (int)hipGetLastError();
}

}  // namespace insr

using namespace insr;

#ifdef INSR_STAMPS
extern "C" int insr_diag_stamps_adv(unsigned long long* host, int n) {
  if (n > 8 * kAdvStamps) n = 8 * kAdvStamps;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_adv_stamps), n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
#endif

extern "C" {

long insr_advect1d_rows(long n_points) {
  if (n_points < 0) return INSR_EINVAL;
  return adv_blocks((n_points + 15) / 16);
}

int insr_advect1d_iteration(const float* params, const float* prev_params, int num_hidden, int width, long n,
                            long n_band_half, const float* box_lo, const float* box_hi, float dt, float vel,
                            float main_total, float bc_total, unsigned long long seed, void* sampler_state,
                            float* points, float* partials, long stride, float* loss_part, float* losses,
                            void* stream) {
  if (width != kAdvW || num_hidden < 1 || num_hidden > 3) return INSR_EWIDTH;  // (LDS: 3 hidden layers)
  if (!params || !prev_params || !box_lo || !box_hi || !sampler_state || !partials || !loss_part || !losses)
    return INSR_EINVAL;
  if (n < 1 || n_band_half < 0 || n + 2 * n_band_half > 0x7fffffffL || !(dt > 0.f) || !(main_total > 0.f) ||
      (n_band_half > 0 && !(bc_total > 0.f)))
    return INSR_EINVAL;
  if (stride < (long)out_off(1, kAdvW, num_hidden) + kAdvW + 1 || (stride & 3)) return INSR_EINVAL;
  AdvectPk pk{};
  pk.prm = params;
  pk.prev = prev_params;
  pk.part = partials;
  pk.lpart = loss_part;
  pk.xout = points;
  pk.state = (unsigned long long*)sampler_state;
  pk.seed = seed;
  pk.stride = stride;
  pk.n = (int)n;
  pk.h = (int)n_band_half;
  const long total = n + 2 * n_band_half;
  pk.tiles = (int)((total + 15) / 16);
  pk.nb = adv_blocks(pk.tiles);
  for (int k = 0; k < 3; ++k) {
    pk.lo[k] = box_lo[k];
    pk.hi[k] = box_hi[k];
  }
  pk.inv_dt = 1.f / dt;
  pk.hvel = 0.5f * vel;
  pk.gmain = 2.f / main_total;
  pk.gbc = n_band_half > 0 ? 2.f / bc_total : 0.f;
  pk.loss = losses;
  pk.smain = 1.f / main_total;
  pk.sbc = n_band_half > 0 ? 1.f / bc_total : 0.f;
  hipStream_t st = (hipStream_t)stream;
  int rc;
  switch (num_hidden) {
    case 1: rc = advect_launch<1>(pk, st); break;
    case 2: rc = advect_launch<2>(pk, st); break;
    default: rc = advect_launch<3>(pk, st); break;
  }
  return rc ? rc : pk.nb;
}

}  // extern "C"
