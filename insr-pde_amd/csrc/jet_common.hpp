// jet_common.hpp -- shared device helpers of the gfx950 SIREN jet kernels.
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
// Layout on the chip ("transposed" orientation: neurons are MFMA rows, 16 points the
// 16 MFMA columns; a lane (g = lane >> 4, c = lane & 15) holds rows 4g..4g+3 of a
// 16-row tile at point c, which is both the MFMA C/D layout and the B-operand layout
// of the next layer):
//   * the forward saves pre-activation streams to HBM in that layout (each store =
//     one contiguous 1 KiB wave write), [layer][16-point tile][stream][row tile][lane][4];
//   * the backward rebuilds sin/cos from the saved z, runs the sine reverse
//     lane-locally and forms dW as an MFMA GEMM over points x streams.
// Kernels: jet_split.hpp (exact fp32 MFMA), jet_x6.hpp (split-bf16, the default),
// jet_x6w.hip (two-kernel backward for wide nets / large batches).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/insr_siren.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define OMEGA 30.0f
#define OMEGA2 900.0f
#define OMEGA3 27000.0f

namespace insr {


// 16-point tiles of the saved-activation layout for n points (padded to 64 points)
__host__ __device__ inline long act_tiles(long n) { return ((n + 63) / 64) * 4; }

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__host__ __device__ inline long hidden_off(int din, int W, int j) {
  // offset of net.{2j}.weight for hidden linear j >= 1
  return (long)W * din + W + (long)(j - 1) * ((long)W * W + W);
}
__host__ __device__ inline long out_off(int din, int W, int L) {
  return (long)W * din + W + (long)L * ((long)W * W + W);
}

// pre-split weight planes after the parameters (INSR_MODE_WSPLIT): orientation o (0: W_j rows,
// the forward's A operand; 1: W_j^T rows, the backward's), layer j - 1, fragment rt (W / 16)
// x kc (W / 32), term q (3), lane: 16 B = 8 bf16 of one term -- 3 L W^2 / 8 u32x4 per
// orientation, 3 L W^2 floats in all
__host__ __device__ inline long wsplit_offset(int din, int dout, int L, int W) {
  return (out_off(din, W, L) + (long)dout * W + dout + 3) & ~3L;
}
__host__ __device__ inline long wsplit_orient_vecs(int L, int W) { return (long)L * W * W * 3 / 8; }
// ... followed by the fp16 planes of the forward orientation (INSR_PREC_F16X3): 2^8 W_j in two
// fp16 terms, [layer][rt][kc][term][lane] 16 B each -- L W^2 floats
constexpr float kF16WScale = 256.0f;  // weights' power-of-two scale in the fp16 planes
__host__ __device__ inline long wsplit_f16_offset(int din, int dout, int L, int W) {
  return wsplit_offset(din, dout, L, W) + 3L * L * W * W;
}
// ... then 2^8 W_j^T likewise (the backward orientation of the fp16 planes: the f16x3 backward's
// propagation A operand) -- 5 L W^2 floats of planes in all
__host__ __device__ inline long wsplit_f16t_offset(int din, int dout, int L, int W) {
  return wsplit_f16_offset(din, dout, L, W) + (long)L * W * W;
}
__host__ __device__ inline long wsplit_f16_vecs(int L, int W) { return (long)L * W * W / 4; }  // u32x4 per fp16 orientation
// ... then one status quad: word 0 != 0 once a hidden weight with |w| >= kF16WMax was split into the fp16
// planes (2^8 w would leave fp16's range: its terms are clamped, so the f16x3 products of that layer are
// not the network's).  Set by wsplit_kernel (cleared by the host launch first) and by the Adam launch
// (sticky); read by insr_siren_wsplit_status.
constexpr float kF16WMax = 255.0f;
__host__ __device__ inline long wsplit_status_offset(int din, int dout, int L, int W) {
  return wsplit_f16t_offset(din, dout, L, W) + (long)L * W * W;
}
__host__ __device__ inline long wsplit_total_floats(int L, int W) { return 5L * L * W * W + 4; }

// wave-tile base of layer `layer` in the saved-activation buffer
// CUs of the current device, queried once (thread-safe function-local static; one device per process)
inline int device_cus() {
  static const int c = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    return (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) ? 256 : v;
  }();
  return c;
}

__device__ __forceinline__ float* act_base(float* act, int layer, int ntiles, int tile, int S, int NT) {
  return act + ((long)layer * ntiles + tile) * (long)(S * NT) * 256;
}
__device__ __forceinline__ const float* act_base(const float* act, int layer, int ntiles, int tile, int S,
                                                 int NT) {
  return act + ((long)layer * ntiles + tile) * (long)(S * NT) * 256;
}

// v + (v of the lane DPP control CTRL selects), in the VALU (no LDS crossbar)
template <int CTRL>
__device__ __forceinline__ float add_dpp(float v) {
  const int o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false);
  return v + __builtin_bit_cast(float, o);
}

// sum over the 16 point-lanes that share lane>>4 (one DPP row), every lane gets it:
// pairs (quad_perm 1,0,3,2), quads (quad_perm 2,3,0,1), halves (row_half_mirror),
// row (row_mirror) -- fixed order, no ds_bpermute round trips
__device__ __forceinline__ float sum16(float v) {
  v = add_dpp<0xB1>(v);
  v = add_dpp<0x4E>(v);
  v = add_dpp<0x141>(v);
  v = add_dpp<0x140>(v);
  return v;
}

// ---------------------------------------------------------------------------
// sin / cos of w*z.  Two-part Cody-Waite reduction by 2 pi (n = rint(x / 2 pi); 6.28125 n is
// exact for |n| < 2^16) to r in [-pi, pi], then the hardware v_sin_f32 / v_cos_f32 on
// r / 2 pi (|r / 2 pi| <= 1/2 revolution, where they are accurate): max abs error 3.8e-7 over
// |x| <= 200 (tools/study/sin_acc.hip on MI355X; the fp32 rounding of the argument w z
// itself is 7.6e-6 there).  5 + 1 (+1 for cos) VALU ops instead of a ~20-op polynomial pair;
// no branches.  Valid for |x| <= 8192; a wave with any larger |x| takes the libm (ocml)
// path instead (uniform branch).
// ---------------------------------------------------------------------------
constexpr float kFastArgMax = 8192.0f;

__device__ __forceinline__ float revs_reduced(float x) {
  const float n = rintf(x * 0.15915494309189535f);
  float r = fmaf(-n, 6.28125f, x);
  r = fmaf(-n, 1.9353071795864769e-3f, r);
  return r * 0.15915494309189535f;  // revolutions in [-1/2, 1/2]
}

__device__ __forceinline__ void sincos_fast(float x, float& s, float& c) {
  const float t = revs_reduced(x);
  s = __builtin_amdgcn_sinf(t);
  c = __builtin_amdgcn_cosf(t);
}

__device__ __forceinline__ float sin_fast(float x) { return __builtin_amdgcn_sinf(revs_reduced(x)); }

// true if any lane of the wave holds an argument outside the fast range
__device__ __forceinline__ bool wave_any_big(float amax) {
  return __any(amax > kFastArgMax);
}

template <int CTRL>
__device__ __forceinline__ float max_dpp(float v) {
  const int o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false);
  return fmaxf(v, __builtin_bit_cast(float, o));
}
// max over the wave's 64 lanes of NON-NEGATIVE values as a wave-uniform (scalar) result: the max of
// each 16-lane row by four DPP steps (as sum16), then the four rows' maxima read into scalars and
// combined as unsigned integers (non-negative floats order like their bit patterns) -- no LDS
// crossbar round trips (__shfl_xor's ds_bpermute chain)
__device__ __forceinline__ float wave_max_nn(float v) {
  v = max_dpp<0xB1>(v);
  v = max_dpp<0x4E>(v);
  v = max_dpp<0x141>(v);
  v = max_dpp<0x140>(v);
  const int b = __builtin_bit_cast(int, v);
  const unsigned r0 = (unsigned)__builtin_amdgcn_readlane(b, 0), r1 = (unsigned)__builtin_amdgcn_readlane(b, 16);
  const unsigned r2 = (unsigned)__builtin_amdgcn_readlane(b, 32), r3 = (unsigned)__builtin_amdgcn_readlane(b, 48);
  const unsigned m01 = r0 > r1 ? r0 : r1, m23 = r2 > r3 ? r2 : r3;
  return __builtin_bit_cast(float, m01 > m23 ? m01 : m23);
}

// max over the wave's 64 lanes (every lane gets it)
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}


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

// ---- saved-stream reads ----
// A forward saves every z-stream of hidden layers 1..L but only the VALUE stream of the first layer
// (when L > 0): its tangent streams are the columns of W_0 and its Laplacian stream is 0 at every
// point (x enters linearly), so readers rebuild them from the parameters (W_0 row-major W x d_in at
// offset 0 of prm) instead of reading (S - 1) / S of that layer's bytes.
__device__ __forceinline__ bool l0_rebuilt(int layer, int L) { return layer == 0 && L > 0; }
template <int S, bool LAP>
__device__ __forceinline__ floatx4 l0_stream(const float* w0, int din, int s, int rt, int lane) {
  if (LAP && s == S - 1) return floatx4{0.f, 0.f, 0.f, 0.f};
  const float* p = w0 + (long)(16 * rt + 4 * (lane >> 4)) * din + (s - 1);
  return floatx4{p[0], p[din], p[2 * din], p[3 * din]};
}
// z-stream s of row tile rt at this lane's point: saved, or rebuilt (l0 = l0_rebuilt(layer, L), s >= 1)
template <int NT, int S, bool LAP>
__device__ __forceinline__ floatx4 load_zs(const float* base, int s, int rt, int lane, bool l0, const float* w0,
                                           int din) {
  if (l0 && s > 0) return l0_stream<S, LAP>(w0, din, s, rt, lane);
  return *reinterpret_cast<const floatx4*>(base + ((s * NT + rt) * 64 + lane) * 4);
}

// h-stream s of a sine layer (for the weight gradient of the layer above),
// rebuilt from saved z-streams + cached sin/cos (l0: the first layer's rebuilt streams, above).
template <int NT, int S, bool LAP>
__device__ __forceinline__ floatx4 h_stream(const float* base, int s, int rt, int lane, const floatx4& sn,
                                            const floatx4& cs, bool l0 = false, const float* w0 = nullptr,
                                            int din = 0) {
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  if (s == 0) return sn;
  const floatx4 zs = load_zs<NT, S, LAP>(base, s, rt, lane, l0, w0, din);
  floatx4 out;
  if (LAP && s == S - 1) {
    floatx4 t2 = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < NTAN; ++i) {
      const floatx4 t = load_zs<NT, S, LAP>(base, 1 + i, rt, lane, l0, w0, din);
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

// As h_stream, and stores the loaded z-stream s (>= 1) into zkeep[s] for the caller's
// next sine reverse (the Laplacian stream reads the tangents from zkeep, which the
// caller fills in stream order 1..S-1 before stream S-1).
template <int NT, int S, bool LAP>
__device__ __forceinline__ floatx4 h_from_z(const float* base, int s, int rt, int lane, const floatx4& sn,
                                            const floatx4& cs, floatx4 (&zkeep)[S], bool l0 = false,
                                            const float* w0 = nullptr, int din = 0) {
  constexpr int NTAN = LAP ? S - 2 : S - 1;
  if (s == 0) return sn;
  const floatx4 zs = load_zs<NT, S, LAP>(base, s, rt, lane, l0, w0, din);
  zkeep[s] = zs;
  floatx4 out;
  if (LAP && s == S - 1) {
    floatx4 t2 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NTAN; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) t2[r] = fmaf(zkeep[1 + i][r], zkeep[1 + i][r], t2[r]);
#pragma unroll
    for (int r = 0; r < 4; ++r) out[r] = OMEGA * cs[r] * zs[r] - OMEGA2 * sn[r] * t2[r];
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) out[r] = OMEGA * cs[r] * zs[r];
  }
  return out;
}

// ---------------------------------------------------------------------------
// Diagnostic phase stamps (build with -DINSR_STAMPS, tools/diag_stamps.py): s_memtime
// at phase boundaries for every wave of two blocks, [blk][wave][layer][phase].
// ---------------------------------------------------------------------------
#ifdef INSR_STAMPS
constexpr int kStampSlots = 2 * 16 * 8 * 8;
static __device__ unsigned long long g_insr_stamps[kStampSlots];
#define INSR_STAMP(layer, k)                                                                      \
  do {                                                                                            \
    const int sb_ = blockIdx.x == 0 ? 0 : (blockIdx.x == gridDim.x / 2 ? 1 : -1);               \
    if (sb_ >= 0 && (threadIdx.x & 63) == 0 && (layer) < 8)                                        \
      g_insr_stamps[((sb_ * 16 + (threadIdx.x >> 6)) * 8 + (layer)) * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define INSR_STAMP(layer, k) \
  do {                       \
  } while (0)
#endif

// ---------------------------------------------------------------------------
// launchers (defined in jet_split_fwd.hip / jet_split_bwd.hip / jet_x6_*.hip / jet_x6w.hip)
// ---------------------------------------------------------------------------
int dispatch_fwd_split(int NT, int S, bool LAP, int T, const float* x, int N, int din, int dout, int L,
                       const float* prm, float* y, float* dy, float* lap, float* act, hipStream_t st);
int dispatch_bwd_split(int NT, int S, bool LAP, int T, const float* x, int N, int din, int dout, int L,
                       const float* prm, const float* act, const float* gy, const float* gdy, const float* glap,
                       float* part, long P, hipStream_t st);
// split-bf16 kernels, per precision NQ (bf16 terms per operand: 3 = x6, 2 = x3, 1 = bf16; 4 = the
// fp16 two-term forward f16x3)
template <int NQ>
int dispatch_fwd_q(int NT, int S, bool LAP, int T, const float* x, int N, int din, int dout, int L,
                   const float* prm, float* y, float* dy, float* lap, float* act, int nbal, hipStream_t st);
constexpr int kFwdJobs = INSR_MAX_FWD_JOBS;
template <int NQ>
int dispatch_fwd_multi_q(int NT, int S, bool LAP, int T, const InsrJetJob* jobs, const int* small, const int* nbal,
                         int njobs, int din, int dout, int L, hipStream_t st);
// A squared-residual loss term's operands (residual.hip, insr_sq_loss_group): a from its first term
struct LossIn {
  const float* a;
  const float* b;
  const float* c;
  const float* d;
  float alpha, beta, gamma, delta;
  long sb = 1, sc = 1, sd = 1;  // element strides of b, c, d
};

// r = alpha (a + beta b) + gamma (c + delta d), evaluated in exactly that order
// (the reference's rounding for (u - u0)/dt + v (ux + u0x)/2 and u - (u_prev - grad_p))
__device__ __forceinline__ float combo_r(const float* a, const float* b, const float* c, const float* d, float alpha,
                                         float beta, float gamma, float delta, long sb, long sc, long sd, long i) {
  float p = a[i];
  if (b) p = p + beta * b[i * sb];
  p = alpha * p;
  if (c) {
    float q = c[i * sc];
    if (d) q = q + delta * d[i * sd];
    p = p + gamma * q;
  }
  return p;
}
__device__ __forceinline__ float combo_residual(const LossIn& in, long i) {
  return combo_r(in.a, in.b, in.c, in.d, in.alpha, in.beta, in.gamma, in.delta, in.sb, in.sc, in.sd, i);
}

// In-kernel adjoint seeds of a reverse jet (include/insr_siren.h InsrSeed): the loss terms that seed
// one adjoint stream of one job, evaluated where the kernel reads that adjoint -- the same
// expressions as sq_loss_group_kernel's gradient, so the seeds are its values bit for bit
struct SeedTerm {
  const float *a, *b, *c, *d;  // a = the stream's output buffer + a_off (the term's first element)
  float alpha, beta, gamma, delta;
  long sb, sc, sd;
  long n, a_off;     // COMBO terms / BANDS rows per band; first element of the term range
  float g2;          // 2 * scale
  int kind, m, job, stream, loss;
};
struct SeedTab {
  SeedTerm t[INSR_SEED_MAX];
  int nt;            // 0: no seeded stream (every adjoint from its pointer)
  float* lpart;      // [block][INSR_SEED_MAX] square sums of the terms each block seeds
};

__device__ __forceinline__ void seed_sq_add(float (&sq)[INSR_SEED_MAX], int k, float v) {
#pragma unroll
  for (int q = 0; q < INSR_SEED_MAX; ++q)
    if (q == k) sq[q] += v;
}

// The adjoint of element e of `stream` of job `job` (0 where no term covers it); count: the lane
// owning the element adds the covering term's square to sq[loss] (one lane per element)
__device__ __forceinline__ float seed_adjoint(const SeedTab& S, int job, int stream, long e, bool count,
                                              float (&sq)[INSR_SEED_MAX]) {
  float g = 0.f;
#pragma unroll
  for (int k = 0; k < INSR_SEED_MAX; ++k) {
    if (k >= S.nt) break;
    const SeedTerm& T = S.t[k];
    if (T.job != job || T.stream != stream) continue;
    const long rel = e - T.a_off;
    if (T.kind == INSR_LOSS_COMBO) {
      if (rel < 0 || rel >= T.n) continue;
      const float r = combo_r(T.a, T.b, T.c, T.d, T.alpha, T.beta, T.gamma, T.delta, T.sb, T.sc, T.sd, rel);
      g = T.alpha * (T.g2 * r);  // sq_loss_group_kernel: cf[0] * (g2 * r)
      if (count) seed_sq_add(sq, T.loss, r * r);
    } else {
      if (rel < 0 || rel >= 2 * T.n * T.m) continue;
      const long row = rel / T.m;
      const int col = (int)(rel - row * T.m);
      if (col != (row < T.n ? 0 : 1)) continue;
      const float v = T.a[rel];
      g = T.g2 * v;
      if (count) seed_sq_add(sq, T.loss, v * v);
    }
  }
  return g;
}

// seed_adjoint in two halves, so a kernel can issue the operand loads early and finish after other work
// (their latency under it): the covering term of element e and its raw operands, then the adjoint (the
// same expressions as combo_r / sq_loss_group_kernel) and its square into sq[loss]
struct SeedOps {
  float a, b, c, d;
  int k;  // the covering term, -1: none (adjoint 0)
};
__device__ __forceinline__ SeedOps seed_gather(const SeedTab& S, int job, int stream, long e) {
  SeedOps v{0.f, 0.f, 0.f, 0.f, -1};
#pragma unroll
  for (int k = 0; k < INSR_SEED_MAX; ++k) {
    if (k >= S.nt) break;
    const SeedTerm& T = S.t[k];
    if (T.job != job || T.stream != stream) continue;
    const long rel = e - T.a_off;
    if (T.kind == INSR_LOSS_COMBO) {
      if (rel < 0 || rel >= T.n) continue;
      v.k = k;
      v.a = T.a[rel];
      if (T.b) v.b = T.b[rel * T.sb];
      if (T.c) v.c = T.c[rel * T.sc];
      if (T.d) v.d = T.d[rel * T.sd];
    } else {
      if (rel < 0 || rel >= 2 * T.n * T.m) continue;
      const long row = rel / T.m;
      const int col = (int)(rel - row * T.m);
      if (col != (row < T.n ? 0 : 1)) continue;
      v.k = k;
      v.a = T.a[rel];
    }
  }
  return v;
}
__device__ __forceinline__ float seed_finish(const SeedTab& S, const SeedOps& v, float (&sq)[INSR_SEED_MAX]) {
  float g = 0.f;
#pragma unroll
  for (int k = 0; k < INSR_SEED_MAX; ++k) {
    if (k >= S.nt) break;
    if (v.k != k) continue;
    const SeedTerm& T = S.t[k];
    if (T.kind == INSR_LOSS_COMBO) {
      float p = v.a;
      if (T.b) p = p + T.beta * v.b;
      p = T.alpha * p;
      if (T.c) {
        float q = v.c;
        if (T.d) q = q + T.delta * v.d;
        p = p + T.gamma * q;
      }
      g = T.alpha * (T.g2 * p);  // sq_loss_group_kernel: cf[0] * (g2 * r)
      seed_sq_add(sq, T.loss, p * p);
    } else {
      g = T.g2 * v.a;
      seed_sq_add(sq, T.loss, v.a * v.a);
    }
  }
  return g;
}

// The block's square sums (sq of every lane of the calling wave, zeros where a lane counted nothing)
// into its loss_part row: a fixed butterfly, lane 0 stores.  Call from one whole wave.
__device__ __forceinline__ void seed_sq_store(const SeedTab& S, float (&sq)[INSR_SEED_MAX], unsigned block) {
#pragma unroll
  for (int q = 0; q < INSR_SEED_MAX; ++q) {
    float v = sq[q];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    sq[q] = v;
  }
  if ((threadIdx.x & 63) == 0) {
    floatx4 r = floatx4{sq[0], sq[1], sq[2], sq[3]};
    *reinterpret_cast<floatx4*>(S.lpart + (long)block * INSR_SEED_MAX) = r;
  }
}

// The loss values of a seeded backward (InsrLossFin) in the sums launch that follows it: one wave,
// lane l sums rows l, l + 64, ... of each column in order, then a fixed butterfly; out[k] leaves as
// an sc1 store acknowledged before the caller's plateau ticket (residual.hip header: the hand-off the
// last block's sc1 load of the loss reads)
struct LossFin {
  const float* part = nullptr;
  int rows = 0, nloss = 0;
  float scale[INSR_SEED_MAX] = {0.f, 0.f, 0.f, 0.f};
  float* out[INSR_SEED_MAX] = {nullptr, nullptr, nullptr, nullptr};
};
__device__ __forceinline__ void loss_finalize(const LossFin& F) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < INSR_SEED_MAX; ++k) {
    if (k >= F.nloss) break;
    float v = 0.f;
    for (int r = lane; r < F.rows; r += 64) v += F.part[(long)r * INSR_SEED_MAX + k];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) __hip_atomic_store(F.out[k], F.scale[k] * v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (lane == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The jobs of one tile-split backward launch: batches of ONE network and jet mode (its weights
// are the launch's), blocks [first[k], first[k + 1]) run job k -- nbal[k] > 0: its tiles balanced
// over that many blocks (T = 3 / 5 shapes), else T-tile blocks.  One job = insr_siren_jet_bwd.
constexpr int kBwdJobs = INSR_MAX_BWD_JOBS;
struct BwdJobsX6 {
  const float* x[kBwdJobs];
  const float* act[kBwdJobs];
  const float* gy[kBwdJobs];
  const float* gdy[kBwdJobs];
  const float* glap[kBwdJobs];
  int n[kBwdJobs];
  int nbal[kBwdJobs];
  int first[kBwdJobs + 1];
  int njobs;
  SeedTab seeds;  // seeds.nt == 0: every adjoint from gy / gdy / glap
};
// jobs == NULL: occupancy query (resident blocks per CU of the instantiation)
template <int NQ>
int dispatch_bwd_q(int NT, int S, bool LAP, int T, const BwdJobsX6* jobs, int din, int dout, int L,
                   const float* prm, float* part, long P, hipStream_t st);
// two-kernel backward (W = 128 / 256): propagation kernel + dW GEMM + reductions (jet_x6w.hpp)
// The Adam (+ plateau) update a sums launch runs as its epilogue (reduce_dw_kernel with m != NULL,
// optim.hpp): the flat parameter buffer and its moments, the optimiser state, the buffer's SIREN shape
// (its weight planes), the plateau loss (NULL: Adam only); t = st[STEP] + 1 either way
struct AdamArgs {
  float* p = nullptr;
  float* m = nullptr;
  float* v = nullptr;
  float* st = nullptr;
  const float* loss = nullptr;
  int patience = 0;
  float b1 = 0.f, b2 = 0.f, eps = 0.f;
  int shape[4] = {0, 0, 0, 0};
  LossFin fin;  // fin.nloss > 0: the sums launch also finishes a seeded backward's loss values
};

struct FbJobs;  // (below) the job table of the two-kernel and jet_fb.hpp backwards
template <int NQ>
int dispatch_wide_bwd_q(int NT, int S, bool LAP, const FbJobs& J, int N, int din, int dout, int L, const float* prm,
                        float* work, float* grad, int accumulate, int f16, int phases, const AdamArgs& A,
                        hipStream_t st);
long wide_work_floats(long n, int din, int dout, int L, int W, int S);
template <int NQ>
int dispatch_fwd_mixed_q(int NT, int din, const InsrJetJob* jobs, const int* modes, const float* scalars, int njobs,
                         int dout, int L, hipStream_t st);
// the pre-split weight planes of (prm, shape) written to `planes` (wsplit_offset floats after prm
// in a params buffer of INSR_MODE_WSPLIT), one launch
int wsplit_launch(const float* prm, int din, int dout, int L, int W, float* planes, hipStream_t st);
void wide_launch_threads(long n, int din, int dout, int L, int W, int S, long* out);
// resident-dW backward (jet_x6r.hpp: W = 128, L <= 4, split-bf16 x6): one persistent launch + the
// fixed-order partial sums
int dispatch_resident_bwd(int S, bool LAP, int L, const float* x, int N, int din, int dout, const float* prm,
                          const float* act, const float* gy, const float* gdy, const float* glap, float* work,
                          float* grad, int accumulate, hipStream_t st);
long resident_work_floats(long n, int din, int dout, int L);
int resident_blocks(long n);

// The jobs of one launch: batches of ONE network (its params), e.g. a phase's interior points and
// its wall bands from separate network calls; job k covers global tiles [tstart[k], tstart[k + 1]).
struct FbJobs {
  const float* x[kBwdJobs];
  const float* act[kBwdJobs];  // the forward's saved streams (the saved-stream variant; unread by recompute)
  const float* gy[kBwdJobs];
  const float* gdy[kBwdJobs];
  const float* glap[kBwdJobs];
  int n[kBwdJobs];
  int tstart[kBwdJobs + 1];
  int njobs;
  SeedTab seeds;  // the saved-stream variant only (the recompute variant takes pointers)
};
constexpr int kFbSeedTiles = 24;  // at most this many tiles per block take in-kernel seeds (staged in LDS)
// recompute backward (jet_fb.hpp: W = 128, L = 4, f16x3 with per-tile scales): ONE persistent launch
// (forward + reverse jet per tile, dW resident per CU) + the fixed-order sums; act is not read
int dispatch_fb_bwd(int S, bool LAP, int L, const FbJobs& J, int din, int dout, const float* prm, float* work,
                    float* grad, int accumulate, int saved, int phases, const AdamArgs& A, hipStream_t st);
bool fb_supported(int S, bool LAP, int L);
bool fb_saved_supported(int S, bool LAP, int L);
long fb_work_floats(long tiles, int din, int dout, int L);
int fb_launch_blocks(long tiles);

// (S, LAP) combinations: value (1), grad d=1..3 (2..4), lap d=1..3 (3..5)
#define INSR_DISPATCH(NTV, FN, ...)                \
  switch (S * 2 + (LAP ? 1 : 0)) {                 \
    case 2: return FN<NTV, 1, false>(__VA_ARGS__); \
    case 4: return FN<NTV, 2, false>(__VA_ARGS__); \
    case 6: return FN<NTV, 3, false>(__VA_ARGS__); \
    case 8: return FN<NTV, 4, false>(__VA_ARGS__); \
    case 7: return FN<NTV, 3, true>(__VA_ARGS__);  \
    case 9: return FN<NTV, 4, true>(__VA_ARGS__);  \
    case 11: return FN<NTV, 5, true>(__VA_ARGS__); \
    default: return INSR_EINVAL;                   \
  }

}  // namespace insr
