// capi.hip -- the C ABI of libinsr_hip.so (include/insr_siren.h): argument checks,
// kernel-variant selection, the partial reducer and the device-resident optimiser.
#include <cstdlib>

#include "jet_common.hpp"

namespace insr {

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

// Kernel-variant choice.  Batches up to these sizes use the tile-split kernels (a
// 16-point tile per 4-wave block, neurons split over the waves); larger ones the
// wave-tile kernels (one wave per 16 points).  Both write/read the same saved-
// activation layout, so forward and backward choose independently.  Defaults from
// tools/kbench.py on MI355X (W=128): the split forward wins at every size
// measured (324..65536 points); the split backward wins at every size for
// derivative jets even counting its 4x larger partial reduction (65536 points, LAP:
// 1187+270 us vs 1793+68 us), but loses beyond 8192 points for value jets (16384:
// 111+69 us vs 144+17 us).
// Env overrides: INSR_SPLIT_MAX_N_FWD / _BWD / _BWD_VALUE (points).
static int g_thr[3] = {-1, -1, -1};  // fwd, bwd (S > 1), bwd value

static int env_or(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

int split_max_n() {
  if (g_thr[0] < 0) {
    g_thr[0] = env_or("INSR_SPLIT_MAX_N_FWD", 1 << 30);
    g_thr[1] = env_or("INSR_SPLIT_MAX_N_BWD", 1 << 30);
    g_thr[2] = env_or("INSR_SPLIT_MAX_N_BWD_VALUE", 8192);
  }
  return g_thr[1];
}

bool use_split_fwd(long n) {
  split_max_n();
  return n <= g_thr[0];
}

bool use_split_bwd(long n, int S) {
  split_max_n();
  return n <= (S == 1 ? g_thr[2] : g_thr[1]);
}

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

bool shape_ok(int din, int dout, int L, int width, int mode) {
  if (din < 1 || din > 3 || dout < 1 || dout > 3 || L < 0 || L > 64) return false;
  if (nt_for(width) < 0) return false;
  const int S = streams_for(din, mode);
  if (S < 1 || S > 4) return false;
  if (mode == INSR_MODE_LAP && din > 2) return false;
  return true;
}

}  // namespace insr

using namespace insr;

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

long insr_jet_partial_bytes(long n, int din, int dout, int L, int W, int mode) {
  return (long)insr_jet_partial_blocks(n, din, mode) * insr_siren_param_count(din, dout, L, W) * (long)sizeof(float);
}

int insr_siren_jet_fwd(const float* x, long n, int din, int dout, int L, int W, int mode, const float* params,
                       float* y, float* dy, float* lap, float* act, void* stream) {
  if (!shape_ok(din, dout, L, W, mode) || n < 0 || n > 0x7fffffffL) return INSR_EINVAL;
  if (n == 0) return 0;
  if (!x || !params || !y) return INSR_EINVAL;
  if (mode != INSR_MODE_VALUE && !dy) return INSR_EINVAL;
  if (mode == INSR_MODE_LAP && !lap) return INSR_EINVAL;
  const int S = streams_for(din, mode);
  const int NT = nt_for(W);
  if (use_split_fwd(n))
    return dispatch_fwd_split(NT, S, mode == INSR_MODE_LAP, x, (int)n, din, dout, L, params, y, dy, lap, act,
                              (hipStream_t)stream);
  return dispatch_fwd_wave(NT, S, mode == INSR_MODE_LAP, x, (int)n, din, dout, L, params, y, dy, lap, act,
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
  const int NT = nt_for(W);
  if (use_split_bwd(n, S))
    return dispatch_bwd_split(NT, S, mode == INSR_MODE_LAP, x, (int)n, din, dout, L, params, act, gy, gdy, glap,
                              partial, P, (hipStream_t)stream);
  return dispatch_bwd_wave(NT, S, mode == INSR_MODE_LAP, x, (int)n, din, dout, L, params, act, gy, gdy, glap,
                           partial, P, (hipStream_t)stream);
}

int insr_jet_partial_blocks(long n, int din, int mode) {
  if (n <= 0) return 0;
  return use_split_bwd(n, streams_for(din, mode)) ? (int)((n + 15) / 16) : (int)((n + kPts - 1) / kPts);
}

int insr_jet_split_threshold(void) { return split_max_n(); }

int insr_jet_set_split_threshold(int n_points) {
  const int old = split_max_n();
  const int v = n_points < 0 ? 0 : n_points;
  g_thr[0] = g_thr[1] = g_thr[2] = v;
  return old;
}

void insr_jet_get_split_thresholds(int* fwd, int* bwd, int* bwd_value) {
  split_max_n();
  if (fwd) *fwd = g_thr[0];
  if (bwd) *bwd = g_thr[1];
  if (bwd_value) *bwd_value = g_thr[2];
}

void insr_jet_set_split_thresholds(int fwd, int bwd, int bwd_value) {
  split_max_n();
  g_thr[0] = fwd < 0 ? 0 : fwd;
  g_thr[1] = bwd < 0 ? 0 : bwd;
  g_thr[2] = bwd_value < 0 ? 0 : bwd_value;
}

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
