// residual.hip -- fused squared-residual losses of the model phases.
//
// The reference writes every PDE residual loss as a chain of aten ops, e.g.
//   torch.mean((u - u_target) ** 2)                       fluid/model.py:96-101
//   torch.mean((div_u - lap_p) ** 2)                       fluid/model.py:121-125
//   torch.mean((u - (u_prev - grad_p)) ** 2)               fluid/model.py:147-151
//   mean(u[:nb, 0] ** 2) + mean(u[nb:, 1] ** 2)  (walls)   fluid/model.py:90-94,129-133
// i.e. 3-5 launches forward and as many backward (sub, pow, mean, slice/select
// backward zero-fills, ...).  On the GPU each of those is a ~3 us launch over a few
// hundred KB, so they cost more than they compute.  Here a loss is ONE launch
// forward (a deterministic reduction in a fixed order) and ONE launch backward (the
// residual is recomputed, every input gradient written in the same pass).  Losses
// over more than 4096 terms combine the per-block partials in the same launch: the
// last block to finish (an atomic ticket) sums them in a fixed order (deterministic)
// and resets the ticket -- no second launch.  Hand-off protocol (block_partial_combine):
// relaxed agent-scope atomic store of the partial (an sc1 store, written through the
// XCD's L2), s_waitcnt vmcnt(0) (the store is acknowledged), relaxed atomicAdd ticket;
// the last block reads the partials with relaxed agent-scope atomic loads (sc1, past
// its L2).  There is NO release/acquire pair: under the HIP memory model this is
// formally a data race; it is correct on gfx950 because the sc1 store completes at the
// coherence point before the waitcnt returns and the sc1 loads read that point
// (MI355X_MICROARCH.md hand-off table row 1).  An acq_rel ticket would add an L2
// write-back + invalidate per block.
#include "jet_common.hpp"

namespace insr {

constexpr int kLossThreads = 512;
constexpr int kLossMaxBlocks = 256;
constexpr long kLossPerBlock = 4096;  // elements per block (8 per thread) before the grid grows

// LossIn / combo_residual: jet_common.hpp (the in-kernel seeds of the reverse jets share them)

__device__ __forceinline__ float loss_term(int kind, const LossIn& in, long n, int m, long i) {
  if (kind == INSR_LOSS_COMBO) {
    const float r = combo_residual(in, i);
    return r * r;
  }
  const float* a = in.a;
  // INSR_LOSS_BANDS: element i < 2n is row i; band 0 (rows < n) uses column 0, band 1 column 1
  const float v = a[i * m + (i < n ? 0 : 1)];
  return v * v;
}

// The block's partial sum (fixed order: wave butterfly, then the waves in order) and, over a
// grid of nblk blocks, the cross-block combine in the same launch: the partial leaves as an sc1
// store, thread 0 waits for it and takes the ticket with a relaxed atomic (no release fence and
// no L2 write-back; correct on gfx950 by the hardware hand-off in the file header, not by the
// HIP memory model); the LAST block's first wave loads every partial with
// sc1 loads in parallel (lane l: partials l, l + 64, ...) and sums them by a fixed butterfly --
// deterministic, and no serial chain of nblk dependent loads.  Leaves the ticket zero.
__device__ __forceinline__ void block_partial_combine(float acc, float* red, int blk, int nblk, float scale,
                                                      float* __restrict__ out, float* __restrict__ wk,
                                                      float* ticket_word) {
  __shared__ int last;
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float part = 0.f;
    for (int k = 0; k < (int)(blockDim.x / 64); ++k) part += red[k];
    if (nblk == 1) {
      out[0] = scale * part;
      last = 0;
    } else {
      __hip_atomic_store(wk + blk, part, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      last = atomicAdd(reinterpret_cast<unsigned*>(ticket_word), 1u) == (unsigned)nblk - 1 ? 1 : 0;
    }
  }
  __syncthreads();
  if (!last || w != 0) return;
  float tot = 0.f;
  for (int q = lane; q < nblk; q += 64) tot += __hip_atomic_load(wk + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int off = 32; off > 0; off >>= 1) tot += __shfl_xor(tot, off);
  if (lane == 0) {
    out[0] = scale * tot;
    atomicExch(reinterpret_cast<unsigned*>(ticket_word), 0u);
  }
}

// work: kLossMaxBlocks partials + one ticket word (zero-initialised; every launch leaves it 0)
__global__ __launch_bounds__(kLossThreads) void sq_loss_fwd_kernel(int kind, LossIn in, long n, int m, float scale,
                                                                   float* __restrict__ out, float* __restrict__ work) {
  // grid == 1: out[0] = scale * sum;  grid > 1: work[block] = partial sum, the last block combines
  __shared__ float red[kLossThreads / 64];
  const long count = kind == INSR_LOSS_COMBO ? n : 2 * n;
  float acc = 0.f;
#pragma unroll 4
  for (long i = (long)blockIdx.x * kLossThreads + threadIdx.x; i < count; i += (long)gridDim.x * kLossThreads)
    acc += loss_term(kind, in, n, m, i);
  // wave reduction (fixed butterfly order), then the block's waves in order
  block_partial_combine(acc, red, (int)blockIdx.x, (int)gridDim.x, scale, out, work, work + kLossMaxBlocks);
}

__global__ __launch_bounds__(256) void sq_loss_bwd_kernel(int kind, LossIn in, long n, int m, float scale,
                                                          const float* __restrict__ gout, float* __restrict__ ga,
                                                          float* __restrict__ gb, float* __restrict__ gc,
                                                          float* __restrict__ gd) {
  const float g2 = 2.f * scale * gout[0];
  if (kind == INSR_LOSS_COMBO) {
    const float ca = in.alpha, cb = in.alpha * in.beta, cc = in.gamma, cd = in.gamma * in.delta;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
      const float g = g2 * combo_residual(in, i);
      if (ga) ga[i] = ca * g;
      if (gb) gb[i] = cb * g;
      if (gc) gc[i] = cc * g;
      if (gd) gd[i] = cd * g;
    }
    return;
  }
  // bands: the full (2n, m) gradient, zero outside the selected columns; with in.b (the second band in a
  // tensor of its own) a's (n, m) gradient (column 0) and b's (n, m) gradient (column 1)
  const long total = (in.b ? 1 : 2) * n * m;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long row = e / m;
    const int col = (int)(e - row * m);
    if (in.b) {
      if (ga) ga[e] = col == 0 ? g2 * in.a[e] : 0.f;
      if (gb) gb[e] = col == 1 ? g2 * in.b[e] : 0.f;
      continue;
    }
    const int sel = row < n ? 0 : 1;
    ga[e] = col == sel ? g2 * in.a[e] : 0.f;
  }
}

// A GROUP of losses (every squared-residual term of a phase iteration) in ONE launch, each
// with the gradient for a unit output seed (the training loop seeds every loss with 1,
// base/baseModel.py:77): blocks [first[k], first[k + 1]) serve loss k.  A loss's blocks
// grid-stride over every element of its gradient buffers -- each thread writes the gradient of
// the terms it sums, zeros outside the loss range (the other rows of a merged jet launch) --
// then the same deterministic reduction as sq_loss_fwd_kernel (last block of the loss combines
// its partials in block order; work slot k = kLossMaxBlocks partials + a ticket).
constexpr long kGroupPerBlock = 1024;  // elements per block of a group loss

struct LossGroup {
  InsrLoss l[INSR_LOSS_GROUP_MAX];
  int first[INSR_LOSS_GROUP_MAX + 1];
  int count;
};

// elements a loss's blocks walk: its terms, and every gradient element it writes (ga: its
// range [ga_lo, ga_hi) walked as e = ga_lo + i)
__device__ __forceinline__ long loss_span(const InsrLoss& L) {
  long span = L.kind == INSR_LOSS_COMBO ? L.n : 2 * L.n;
  const long lens[4] = {L.ga ? L.ga_hi - L.ga_lo : 0, L.gb ? L.gb_len : 0, L.gc ? L.gc_len : 0, L.gd ? L.gd_len : 0};
  for (int k = 0; k < 4; ++k) span = lens[k] > span ? lens[k] : span;
  return span;
}

__global__ __launch_bounds__(kLossThreads) void sq_loss_group_kernel(const LossGroup G, float* __restrict__ work) {
  __shared__ float red[kLossThreads / 64];
  int k = 0;
#pragma unroll
  for (int q = 1; q < INSR_LOSS_GROUP_MAX; ++q) k += (q < G.count && (int)blockIdx.x >= G.first[q]) ? 1 : 0;
  const InsrLoss& L = G.l[k];
  const int blk = blockIdx.x - G.first[k], nblk = G.first[k + 1] - G.first[k];
  const LossIn in{L.a + L.a_off, L.b, L.c, L.d, L.alpha, L.beta, L.gamma, L.delta, L.sb, L.sc, L.sd};
  const long n = L.n;
  const int m = L.m;
  const float g2 = 2.f * L.scale;
  const float cf[4] = {L.alpha, L.alpha * L.beta, L.gamma, L.gamma * L.delta};
  float* const gp[4] = {L.ga, L.gb, L.gc, L.gd};
  const long gl[4] = {L.ga_hi - L.ga_lo, L.gb_len, L.gc_len, L.gd_len};
  const long span = loss_span(L);
  const long count = L.kind == INSR_LOSS_COMBO ? n : 2 * n;
  float acc = 0.f;
  for (long e = (long)blk * kLossThreads + threadIdx.x; e < span; e += (long)nblk * kLossThreads) {
    if (L.kind == INSR_LOSS_COMBO) {
      float r = 0.f;
      if (e < n) {
        r = combo_residual(in, e);
        acc += r * r;
      }
      const float g = g2 * r;
      if (gp[0] && e < gl[0]) {  // a: element ea = ga_lo + e; the loss range starts at a_off
        const long ea = L.ga_lo + e, t = ea - L.a_off;
        gp[0][ea] = (t >= 0 && t < n) ? cf[0] * (t == e ? g : g2 * combo_residual(in, t)) : 0.f;
      }
#pragma unroll
      for (int q = 1; q < 4; ++q)
        if (gp[q] && e < gl[q]) gp[q][e] = e < n ? cf[q] * g : 0.f;
    } else {  // BANDS: element e of a's gradient; term (row) e of the loss.  With L.b the second band is
              // rows [0, n) of b's own (n, m) tensor (column 1), and b's full gradient is written too
      const float* bb = L.b;
      if (e < count) {
        const float v = (bb && e >= n) ? bb[(e - n) * m + 1] : in.a[e * m + (e < n ? 0 : 1)];
        acc += v * v;
      }
      if (gp[0] && e < gl[0]) {
        const long ea = L.ga_lo + e;
        const long row = ea / m - L.a_off / m;
        const int col = (int)(ea % m);
        const bool hit = row >= 0 && row < (bb ? n : 2 * n) && col == (row < n ? 0 : 1);
        gp[0][ea] = hit ? g2 * in.a[row * m + col] : 0.f;
      }
      if (gp[1] && e < gl[1]) {
        const long row = e / m;
        gp[1][e] = (row < n && e - row * m == 1) ? g2 * bb[e] : 0.f;
      }
    }
  }
  float* wk = work + (long)k * (kLossMaxBlocks + 1);
  block_partial_combine(acc, red, blk, nblk, L.scale, L.out, wk, wk + kLossMaxBlocks);
}

// out = clamp(x + alpha y, lo, hi): the semi-Lagrangian foot of the fluid advection,
// clamp(x - dt u_prev(x), -1, 1) (fluid/model.py:97), one launch instead of add + clamp
__global__ __launch_bounds__(256) void axpy_clamp_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                         float alpha, float lo, float hi, float* __restrict__ out,
                                                         long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    out[i] = fminf(fmaxf(fmaf(alpha, y[i], x[i]), lo), hi);
}

}  // namespace insr

using namespace insr;

extern "C" {

// partials + ticket per group slot (slot 0 is the single-loss kernels' layout)
long insr_sq_loss_work_floats(void) { return (long)INSR_LOSS_GROUP_MAX * (kLossMaxBlocks + 1); }

int insr_sq_loss_fwd(int kind, const float* a, const float* b, const float* c, const float* d, long n, int m,
                     float alpha, float beta, float gamma, float delta, float scale, float* out, float* work,
                     void* stream) {
  if (!a || !out || n < 0) return INSR_EINVAL;
  if (kind == INSR_LOSS_BANDS && (m < 2 || b || c || d)) return INSR_EINVAL;
  if (kind != INSR_LOSS_COMBO && kind != INSR_LOSS_BANDS) return INSR_EINVAL;
  if (d && !c) return INSR_EINVAL;
  const long count = kind == INSR_LOSS_COMBO ? n : 2 * n;
  long nb = (count + kLossPerBlock - 1) / kLossPerBlock;
  if (nb < 1) nb = 1;
  if (nb > kLossMaxBlocks) nb = kLossMaxBlocks;
  if (nb > 1 && !work) return INSR_EINVAL;
  const LossIn in{a, b, c, d, alpha, beta, gamma, delta};
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sq_loss_fwd_kernel, dim3((unsigned)nb), dim3(kLossThreads), 0, st, kind, in, n, m, scale, out,
                     work);
  return (int)hipGetLastError();
}

int insr_axpy_clamp(const float* x, const float* y, float alpha, float lo, float hi, float* out, long n, void* stream) {
  if (!x || !y || !out || n < 0) return INSR_EINVAL;
  if (n == 0) return 0;
  long nb = (n + 255) / 256;
  if (nb > 2048) nb = 2048;
  hipLaunchKernelGGL(axpy_clamp_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, x, y, alpha, lo, hi, out,
                     n);
  return (int)hipGetLastError();
}

int insr_sq_loss_group(const InsrLoss* losses, int count, float* work, void* stream) {
  if (!losses || count < 1 || count > INSR_LOSS_GROUP_MAX) return INSR_EINVAL;
  LossGroup G;
  G.count = count;
  G.first[0] = 0;
  bool multi = false;
  for (int k = 0; k < count; ++k) {
    const InsrLoss& L = losses[k];
    if (!L.a || !L.out || L.n < 0 || L.a_off < 0 || L.ga_lo < 0 || (L.ga && L.ga_hi < L.ga_lo)) return INSR_EINVAL;
    if (L.sb < 1 || L.sc < 1 || L.sd < 1) return INSR_EINVAL;
    if (L.kind != INSR_LOSS_COMBO && L.kind != INSR_LOSS_BANDS) return INSR_EINVAL;
    // BANDS: b (optional) = the second band's own tensor, n x m like a's band (no stride), gb its gradient
    if (L.kind == INSR_LOSS_BANDS && (L.m < 2 || L.c || L.d || L.gc || L.gd || L.a_off % L.m || (L.gb && !L.b) ||
                                      (L.b && L.sb != 1) || (L.gb && L.gb_len > L.n * L.m)))
      return INSR_EINVAL;
    if (L.d && !L.c) return INSR_EINVAL;
    G.l[k] = L;
    long span = L.kind == INSR_LOSS_COMBO ? L.n : 2 * L.n;
    const long lens[4] = {L.ga ? L.ga_hi - L.ga_lo : 0, L.gb ? L.gb_len : 0, L.gc ? L.gc_len : 0, L.gd ? L.gd_len : 0};
    for (int q = 0; q < 4; ++q) span = lens[q] > span ? lens[q] : span;
    long nb = (span + kGroupPerBlock - 1) / kGroupPerBlock;
    if (nb < 1) nb = 1;
    if (nb > kLossMaxBlocks) nb = kLossMaxBlocks;
    multi = multi || nb > 1;
    G.first[k + 1] = G.first[k] + (int)nb;
  }
  for (int k = count + 1; k <= INSR_LOSS_GROUP_MAX; ++k) G.first[k] = G.first[count];
  if (multi && !work) return INSR_EINVAL;
  hipLaunchKernelGGL(sq_loss_group_kernel, dim3((unsigned)G.first[count]), dim3(kLossThreads), 0, (hipStream_t)stream,
                     G, work);
  return (int)hipGetLastError();
}

int insr_sq_loss_bwd(int kind, const float* a, const float* b, const float* c, const float* d, long n, int m,
                     float alpha, float beta, float gamma, float delta, float scale, const float* gout, float* ga,
                     float* gb, float* gc, float* gd, void* stream) {
  if (!a || !gout || n < 0) return INSR_EINVAL;
  if (kind == INSR_LOSS_BANDS && (m < 2 || (!ga && !gb) || (gb && !b) || (!b && !ga) || c || d || gc || gd))
    return INSR_EINVAL;
  if (kind != INSR_LOSS_COMBO && kind != INSR_LOSS_BANDS) return INSR_EINVAL;
  if (d && !c) return INSR_EINVAL;
  const long total = kind == INSR_LOSS_COMBO ? n : (b ? 1 : 2) * n * m;
  if (total == 0) return 0;
  long nb = (total + 255) / 256;
  if (nb > 2048) nb = 2048;
  const LossIn in{a, b, c, d, alpha, beta, gamma, delta};
  hipLaunchKernelGGL(sq_loss_bwd_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, kind, in, n, m, scale,
                     gout, ga, gb, gc, gd);
  return (int)hipGetLastError();
}

}  // extern "C"
