// optim.hpp -- the device side of the Adam + ReduceLROnPlateau update (torch's op order), shared by
// the optimiser launches of capi.hip and the sums + Adam epilogue of reduce_dw_kernel (jet_x6w.hpp):
// one element update, the weight-plane rewrite of an updated hidden weight, the plateau step and
// its last-block ticket.  Reference: base/baseModel.py:55-62,79-81 (Adam, ReduceLROnPlateau).
#pragma once
#include "jet_common.hpp"

namespace insr {

// plateau scheduler step of one device state (torch ReduceLROnPlateau.step after Adam.step)
__device__ void plateau_update(float* st, const float* loss, int patience, int advance_step) {
  if (advance_step) st[INSR_OPT_STEP] = st[INSR_OPT_STEP] + 1.f;
  if (!loss) return;  // advance-only (optimiser without a scheduler)
  // an sc1 load: the loss may come from this launch's own finishing block (jet_common.hpp loss_finalize)
  const float cur = __hip_atomic_load(loss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// The plateau step after every block's Adam update, run by the last block to finish: a two-level
// ticket -- block b adds to shard b % 8, the last adder of a shard (it knows the shard's block count)
// adds to the top word, the last of those runs the step and zeroes all nine words (every block has
// added by then); one word would serialise all the blocks' atomics.  Call with all of the block's
// threads after their last read of st's lr / t.
__device__ __forceinline__ void plateau_after_blocks(float* st, const float* loss, int patience, unsigned bid,
                                                     unsigned nb) {
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* top = reinterpret_cast<unsigned*>(st + INSR_OPT_TICKET);
    unsigned* shard = reinterpret_cast<unsigned*>(st + INSR_OPT_TICKET_SHARDS);
    const unsigned s = bid & 7u;
    const unsigned in_shard = (nb - s + 7u) / 8u, shards = nb < 8u ? nb : 8u;
    if (atomicAdd(shard + s, 1u) == in_shard - 1u && atomicAdd(top, 1u) == shards - 1u) {
      plateau_update(st, loss, patience, 1);
      for (int q = 0; q < 8; ++q) atomicExch(shard + q, 0u);
      atomicExch(top, 0u);
    }
  }
}

// One Adam element in torch's op order (m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
// p.addcdiv_(m, sqrt(v)/sqrt(1-b2^t) + eps, -step_size)) with every multiply-add spelled out, so
// the launches that run it (adam_multi_kernel, reduce_adam_kernel) round identically whatever the
// compiler's contraction choices around them
__device__ __forceinline__ float adam_elem(float g, float m0, float v0, float p0, float step_size, float bc2s,
                                           float w1, float w2, float b2, float eps, float& mi, float& vi) {
  mi = fmaf(w1, g - m0, m0);
  vi = fmaf(w2 * g, g, v0 * b2);
  const float denom = __fadd_rn(__fdiv_rn(sqrtf(vi), bc2s), eps);
  return fmaf(-step_size, __fdiv_rn(mi, denom), p0);
}

// the updated hidden weight (layer j, row n, column m) of a buffer with pre-split planes:
// its three bf16 terms (jet_x6.hpp split, element-wise identical to wsplit_kernel) stored
// into both fragment orientations (jet_common.hpp wsplit_offset) -- the planes stay current
// without a launch of their own
__device__ __forceinline__ void adam_wsplit(float* base, const int (&sh)[4], long i, float w) {
  const int din = sh[0], dout = sh[1], L = sh[2], W = sh[3];
  const long off = i - ((long)W * din + W);
  const long per = (long)W * W + W;
  if (off < 0 || off >= (long)L * per) return;
  const long r = off % per;
  if (r >= (long)W * W) return;  // a bias
  const int j = 1 + (int)(off / per), n = (int)(r / W), m = (int)(r % W);
  const int NT = W / 16, KC = W / 32;
  unsigned short t[3];
  {
    const __bf16 h = (__bf16)w;
    float rs = w - (float)h;
    const __bf16 md = (__bf16)rs;
    rs -= (float)md;
    const __bf16 lo = (__bf16)rs;
    t[0] = __builtin_bit_cast(unsigned short, h);
    t[1] = __builtin_bit_cast(unsigned short, md);
    t[2] = __builtin_bit_cast(unsigned short, lo);
  }
  unsigned short* pl = reinterpret_cast<unsigned short*>(base + wsplit_offset(din, dout, L, W));
  const long ov = wsplit_orient_vecs(L, W) * 8;  // u16 per orientation
  // orientation 0: A row n, k = m; orientation 1: A row m (W^T), k = n
  const int rr[2] = {n, m}, kk[2] = {m, n};
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const int rt = rr[o] >> 4, c = rr[o] & 15, kc = kk[o] >> 5, g = (kk[o] & 31) >> 3, jj = kk[o] & 7;
    const long fr = (((long)(j - 1) * NT + rt) * KC + kc) * 3;
#pragma unroll
    for (int q = 0; q < 3; ++q) pl[o * ov + ((fr + q) * 64 + 16 * g + c) * 8 + jj] = t[q];
  }
  // the fp16 planes (INSR_PREC_F16X3): 2^8 w in two fp16 terms, orientation 0 then 1; a weight outside
  // their range is flagged in the status word (insr_siren_wsplit_status) and clamped there
  unsigned short* ph = reinterpret_cast<unsigned short*>(base + wsplit_f16_offset(din, dout, L, W));
  if (!(fabsf(w) < kF16WMax)) {
    atomicOr(reinterpret_cast<unsigned*>(base + wsplit_status_offset(din, dout, L, W)), 1u);
    w = fminf(fmaxf(w, -kF16WMax), kF16WMax);
  }
  const float ws = w * kF16WScale;
  const _Float16 hh = (_Float16)ws, hl = (_Float16)(ws - (float)hh);
  const long oh = 2L * L * W * W;  // u16 per fp16 orientation
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const int rt = rr[o] >> 4, c = rr[o] & 15, kc = kk[o] >> 5, g = (kk[o] & 31) >> 3, jj = kk[o] & 7;
    const long fr = (((long)(j - 1) * NT + rt) * KC + kc) * 2;
    ph[o * oh + (fr * 64 + 16 * g + c) * 8 + jj] = __builtin_bit_cast(unsigned short, hh);
    ph[o * oh + ((fr + 1) * 64 + 16 * g + c) * 8 + jj] = __builtin_bit_cast(unsigned short, hl);
  }
}

// One launch over up to INSR_ADAM_MAX_TENSORS flat buffers.  The step t used is
// st[STEP] + step_offset (the plateau kernel advances st[STEP] after the update,
// so the bias corrections need no separate prepare launch); torch's op order:
//   m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
//   p.addcdiv_(m, sqrt(v)/sqrt(1-b2^t) + eps, -lr/(1-b1^t))
// b^n in double by repeated squaring: t is integer-valued, and the bias corrections need ~1e-15
// relative, not libm's pow (whose double-precision log / exp chain sat at the head of every block)
__device__ __forceinline__ void powi2_d(double b1, double b2, unsigned n, double& p1, double& p2) {
  p1 = 1.0;
  p2 = 1.0;
  while (n) {
    if (n & 1u) {
      p1 *= b1;
      p2 *= b2;
    }
    b1 *= b1;
    b2 *= b2;
    n >>= 1;
  }
}

}  // namespace insr
