// sampler.hip -- the collocation draws of one phase iteration in ONE launch.
//
// The reference draws its points with torch.rand (base/sampling.py:14-64): the interior
// batch, then every boundary band on its own (rand * (hi - lo) + lo per coordinate).  On the
// GPU each of those is a ~3 us launch over a few KB.  Here every box of one iteration -- the
// interior [-1, 1)^d and the four half-width-eps bands of fluid/model.py:90-94,116-120 --
// comes from one counter-based Philox-4x32-10 stream (the generator cuRAND/rocRAND and
// torch use): value v of the launch = Philox(key = seed, counter = base + v / 4)[v % 4],
// mapped to [lo, hi) as lo + (hi - lo) * u, u = (bits >> 8) * 2^-24 (torch's float uniform).
// The stream position `base` lives on the device and the launch advances it itself (the
// last block to finish, by an atomic ticket), so a captured hipGraph draws fresh points on
// every replay.  Same distributions as the reference; a different stream order (its CPU
// samplers are bit-identical to the reference's and the parity tests pass explicit points).
#include "jet_common.hpp"

namespace insr {

constexpr int kSampThreads = 256;

struct BoxesPk {
  InsrBox box[INSR_MAX_BOXES];
  long first[INSR_MAX_BOXES + 1];  // first value (point * dim + coordinate) of each box
  long rep_stride[INSR_MAX_BOXES];  // floats between repetitions of a box's output
  long per_rep;                     // values of one repetition (first[nbox])
  long per_rep_pad;                 // ... rounded up to whole Philox groups of 4: repetition r starts at
                                    // counter base + r ceil(per_rep / 4), exactly where the r-th of
                                    // reps single launches would start (bit-identical draws)
  int nbox;
  int dim;
  unsigned long long seed;
};

__device__ __forceinline__ uint4 philox4x32_10(unsigned long long key, unsigned long long ctr) {
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

// state[0] = stream position (Philox counter), state[1] (low 32 bits) = the launch's ticket
__global__ __launch_bounds__(kSampThreads) void sample_boxes_kernel(const BoxesPk pk, long total,
                                                                    unsigned long long* __restrict__ state) {
  const unsigned long long base = state[0];
  const long gt = (long)blockIdx.x * kSampThreads + threadIdx.x;
  const long v0 = gt * 4;
  if (v0 < total) {
    const uint4 r = philox4x32_10(pk.seed, base + (unsigned long long)gt);
    const unsigned bits[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long v = v0 + q;
      if (v >= total) break;
      const long rep = v / pk.per_rep_pad, vr = v - rep * pk.per_rep_pad;  // repetition, value within it
      if (vr >= pk.per_rep) continue;  // the padding of a repetition's last Philox group
      int k = 0;
#pragma unroll
      for (int b = 1; b < INSR_MAX_BOXES; ++b) k += (b < pk.nbox && vr >= pk.first[b]) ? 1 : 0;
      const long local = vr - pk.first[k];
      const int j = (int)(local % pk.dim);
      const float u = (float)(bits[q] >> 8) * 5.9604644775390625e-8f;  // 2^-24
      const float lo = pk.box[k].lo[j], hi = pk.box[k].hi[j];
      pk.box[k].out[rep * pk.rep_stride[k] + local] = lo + (hi - lo) * u;
    }
  }
  __syncthreads();  // every thread of this block has read `base`
  if (threadIdx.x == 0) {
    unsigned* ticket = reinterpret_cast<unsigned*>(state + 1);
    if (atomicAdd(ticket, 1u) == gridDim.x - 1) {  // last block: every block has read `base`
      state[0] = base + (unsigned long long)((total + 3) / 4);
      atomicExch(ticket, 0u);
    }
  }
}

}  // namespace insr

using namespace insr;

extern "C" {

long insr_sampler_state_bytes(void) { return 2 * (long)sizeof(unsigned long long); }

int insr_sample_boxes_rep(const InsrBox* boxes, int n_boxes, int dim, int reps, const long* rep_strides,
                          unsigned long long seed, void* state, void* stream) {
  if (!boxes || !state || n_boxes < 1 || n_boxes > INSR_MAX_BOXES || dim < 1 || dim > 3 || reps < 1) return INSR_EINVAL;
  if (reps > 1 && !rep_strides) return INSR_EINVAL;
  BoxesPk pk{};
  long total = 0;
  for (int k = 0; k < n_boxes; ++k) {
    if (boxes[k].n < 0 || (boxes[k].n > 0 && !boxes[k].out)) return INSR_EINVAL;
    // repetitions must not overlap the box's own rows (a stride below n * dim would)
    if (reps > 1 && boxes[k].n > 0 && rep_strides[k] < boxes[k].n * dim) return INSR_EINVAL;
    pk.box[k] = boxes[k];
    pk.first[k] = total;
    pk.rep_stride[k] = reps > 1 ? rep_strides[k] : 0;
    total += boxes[k].n * dim;
  }
  pk.first[n_boxes] = total;
  pk.per_rep = total;
  pk.per_rep_pad = (total + 3) / 4 * 4;
  pk.nbox = n_boxes;
  pk.dim = dim;
  pk.seed = seed;
  if (total == 0) return 0;
  const long all = pk.per_rep_pad * reps;
  const long threads = (all + 3) / 4;
  const long nb = (threads + kSampThreads - 1) / kSampThreads;
  if (nb > 0x7fffffffL) return INSR_EINVAL;
  hipLaunchKernelGGL(sample_boxes_kernel, dim3((unsigned)nb), dim3(kSampThreads), 0, (hipStream_t)stream, pk, all,
                     (unsigned long long*)state);
  return (int)hipGetLastError();
}

int insr_sample_boxes(const InsrBox* boxes, int n_boxes, int dim, unsigned long long seed, void* state,
                      void* stream) {
  return insr_sample_boxes_rep(boxes, n_boxes, dim, 1, nullptr, seed, state, stream);
}

}  // extern "C"
