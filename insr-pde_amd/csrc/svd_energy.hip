// svd_energy.hip -- fused singular-value energies of the elasticity model.
//
// The reference takes the SVD of every deformation gradient J = dq/dx with
// torch.svd (elasticity/model.py:143-144) and only uses the singular values:
//   arap    r_a * sum_points sum_i (s_i - 1)^2          (elasticity/model.py:146-149)
//   volume  r_v * sum_points (prod_i s_i - 1)^2         (elasticity/model.py:160-163)
// Its backward is torch.svd's: dE/dJ = U diag(dE/ds) V^T per point.  On the GPU
// that is a batched-solver launch sequence plus a dozen elementwise launches; here
// one thread owns one point, the SVD is computed in registers and the energy is
// reduced in a fixed order (forward), or the gradient written (backward, SVD
// recomputed -- cheaper than storing U, V).
//   2x2: closed form.  With E=(a+d)/2, F=(a-d)/2, G=(c+b)/2, H=(c-b)/2,
//        Q=|(E,H)|, R=|(F,G)|: s1 = Q+R, s2 = |Q-R|; dQ, dR in closed form
//        (1e-30 guard under the roots, as pde/svd.py).
//   3x3: one-sided (Hestenes) Jacobi on the columns of J: J V -> orthogonal columns,
//        s_i = column norms, u_i = column / s_i; fixed 6 sweeps (quadratic
//        convergence: fp32-exact for these 3x3 blocks); no squaring of J^T J, so
//        small singular values keep their relative accuracy.
#include "jet_common.hpp"

namespace insr {

constexpr int kSvdThreads = 256;
constexpr int kSvdMaxBlocks = 256;

// per-point energy e(s) and de/ds
template <int D>
__device__ __forceinline__ float svd_e(const float (&s)[D], float ra, float rv, float (&de)[D]) {
  float prod = 1.f;
#pragma unroll
  for (int i = 0; i < D; ++i) prod *= s[i];
  float e = 0.f;
#pragma unroll
  for (int i = 0; i < D; ++i) {
    e += ra * (s[i] - 1.f) * (s[i] - 1.f);
    float others = 1.f;
#pragma unroll
    for (int k = 0; k < D; ++k)
      if (k != i) others *= s[k];
    de[i] = 2.f * ra * (s[i] - 1.f) + 2.f * rv * (prod - 1.f) * others;
  }
  e += rv * (prod - 1.f) * (prod - 1.f);
  return e;
}

// 2x2 closed form: singular values (descending, non-negative like torch.svd)
__device__ __forceinline__ void svd2(const float* J, float (&s)[2]) {
  const float a = J[0], b = J[1], c = J[2], d = J[3];
  const float E = (a + d) * 0.5f, F = (a - d) * 0.5f, G = (c + b) * 0.5f, H = (c - b) * 0.5f;
  const float Q = sqrtf(E * E + H * H + 1e-30f), R = sqrtf(F * F + G * G + 1e-30f);
  s[0] = Q + R;
  s[1] = fabsf(Q - R);
}

// d(g0 s1 + g1 s2)/dJ for the 2x2 closed form (|.| has derivative 0 at 0, like torch)
__device__ __forceinline__ void grad2(const float* J, float g0, float g1, float* out) {
  const float a = J[0], b = J[1], c = J[2], d = J[3];
  const float E = (a + d) * 0.5f, F = (a - d) * 0.5f, G = (c + b) * 0.5f, H = (c - b) * 0.5f;
  const float Q = sqrtf(E * E + H * H + 1e-30f), R = sqrtf(F * F + G * G + 1e-30f);
  const float diff = Q - R;
  const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
  // d/dQ and d/dR of g0 s1 + g1 s2
  const float wQ = g0 + g1 * sg, wR = g0 - g1 * sg;
  const float qE = wQ * E / Q, qH = wQ * H / Q, rF = wR * F / R, rG = wR * G / R;
  // E=(a+d)/2, F=(a-d)/2, G=(c+b)/2, H=(c-b)/2
  out[0] = 0.5f * (qE + rF);   // d/da
  out[1] = 0.5f * (rG - qH);   // d/db
  out[2] = 0.5f * (rG + qH);   // d/dc
  out[3] = 0.5f * (qE - rF);   // d/dd
}

// 3x3 one-sided Jacobi: on return B = J V (orthogonal columns), V orthogonal
__device__ __forceinline__ void jacobi3(const float* J, float (&B)[3][3], float (&V)[3][3]) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      B[r][k] = J[r * 3 + k];
      V[r][k] = r == k ? 1.f : 0.f;
    }
#pragma unroll
  for (int sweep = 0; sweep < 6; ++sweep) {
#pragma unroll
    for (int pq = 0; pq < 3; ++pq) {
      const int p = pq == 2 ? 1 : 0, q = pq == 0 ? 1 : 2;
      float alpha = 0.f, beta = 0.f, gamma = 0.f;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        alpha = fmaf(B[r][p], B[r][p], alpha);
        beta = fmaf(B[r][q], B[r][q], beta);
        gamma = fmaf(B[r][p], B[r][q], gamma);
      }
      if (fabsf(gamma) <= 1e-30f) continue;
      const float zeta = (beta - alpha) / (2.f * gamma);
      const float t = copysignf(1.f, zeta) / (fabsf(zeta) + sqrtf(fmaf(zeta, zeta, 1.f)));
      const float cs = 1.f / sqrtf(fmaf(t, t, 1.f)), sn = cs * t;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const float bp = B[r][p], bq = B[r][q];
        B[r][p] = cs * bp - sn * bq;
        B[r][q] = sn * bp + cs * bq;
        const float vp = V[r][p], vq = V[r][q];
        V[r][p] = cs * vp - sn * vq;
        V[r][q] = sn * vp + cs * vq;
      }
    }
  }
}

// singular values = column norms of B; columns of B and V sorted descending in place
// (branch-free compare-and-swap: no dynamic register indexing)
__device__ __forceinline__ void cswap_cols(float (&B)[3][3], float (&V)[3][3], float (&n)[3], int i, int k) {
  const bool sw = n[i] < n[k];
  const float ni = n[i], nk = n[k];
  n[i] = sw ? nk : ni;
  n[k] = sw ? ni : nk;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const float bi = B[r][i], bk = B[r][k], vi = V[r][i], vk = V[r][k];
    B[r][i] = sw ? bk : bi;
    B[r][k] = sw ? bi : bk;
    V[r][i] = sw ? vk : vi;
    V[r][k] = sw ? vi : vk;
  }
}

__device__ __forceinline__ void svd3_sorted(float (&B)[3][3], float (&V)[3][3], float (&s)[3]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) s[k] = sqrtf(B[0][k] * B[0][k] + B[1][k] * B[1][k] + B[2][k] * B[2][k]);
  cswap_cols(B, V, s, 0, 1);
  cswap_cols(B, V, s, 1, 2);
  cswap_cols(B, V, s, 0, 1);
}

// d(sum_k g de_k s_k)/dJ = g U diag(de) V^T for the 3x3 Jacobi SVD (B = J V, sorted).
// U columns: u_k = B[:, k] / s_k; a (near-)zero smallest singular value takes u_0 x u_1,
// signed so that det(U) det(V) = sign det(J)
__device__ __forceinline__ void grad3(const float* Ji, const float (&B)[3][3], const float (&V)[3][3],
                                      const float (&s)[3], float go, const float (&de)[3], float* out) {
  float U[3][3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float inv = s[k] > 1e-30f ? 1.f / s[k] : 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r) U[r][k] = B[r][k] * inv;
  }
  if (!(s[2] > 1e-6f * s[0])) {
    float cx = U[1][0] * U[2][1] - U[2][0] * U[1][1];
    float cy = U[2][0] * U[0][1] - U[0][0] * U[2][1];
    float cz = U[0][0] * U[1][1] - U[1][0] * U[0][1];
    const float detJ = Ji[0] * (Ji[4] * Ji[8] - Ji[5] * Ji[7]) - Ji[1] * (Ji[3] * Ji[8] - Ji[5] * Ji[6]) +
                       Ji[2] * (Ji[3] * Ji[7] - Ji[4] * Ji[6]);
    const float detV = V[0][0] * (V[1][1] * V[2][2] - V[2][1] * V[1][2]) -
                       V[1][0] * (V[0][1] * V[2][2] - V[2][1] * V[0][2]) +
                       V[2][0] * (V[0][1] * V[1][2] - V[1][1] * V[0][2]);
    const float sgn = (detJ < 0.f) == (detV < 0.f) ? 1.f : -1.f;
    U[0][2] = sgn * cx;
    U[1][2] = sgn * cy;
    U[2][2] = sgn * cz;
  }
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int col = 0; col < 3; ++col) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) v = fmaf(U[r][k] * de[k], V[col][k], v);
      out[r * 3 + col] = go * v;
    }
}

__global__ __launch_bounds__(kSvdThreads) void svd_energy_fwd_kernel(const float* __restrict__ J, long n, int d,
                                                                     float ra, float rv, float* __restrict__ out) {
  __shared__ float red[kSvdThreads / 64];
  float acc = 0.f;
  for (long i = (long)blockIdx.x * kSvdThreads + threadIdx.x; i < n; i += (long)gridDim.x * kSvdThreads) {
    if (d == 2) {
      float s[2], de[2];
      svd2(J + i * 4, s);
      acc += svd_e<2>(s, ra, rv, de);
    } else {
      float B[3][3], V[3][3], s[3], de[3];
      jacobi3(J + i * 9, B, V);
      svd3_sorted(B, V, s);
      acc += svd_e<3>(s, ra, rv, de);
    }
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = acc;
  __syncthreads();
  if (threadIdx.x != 0) return;
  float part = 0.f;
  for (int k = 0; k < kSvdThreads / 64; ++k) part += red[k];
  out[blockIdx.x] = part;
}

__global__ __launch_bounds__(64) void svd_combine_kernel(const float* __restrict__ part, int nb,
                                                         float* __restrict__ out) {
  float acc = 0.f;
  for (int k = threadIdx.x; k < nb; k += 64) acc += part[k];
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if (threadIdx.x == 0) out[0] = acc;
}

__global__ __launch_bounds__(kSvdThreads) void svd_energy_bwd_kernel(const float* __restrict__ J, long n, int d,
                                                                     float ra, float rv,
                                                                     const float* __restrict__ gout,
                                                                     float* __restrict__ gJ) {
  const float go = gout[0];
  for (long i = (long)blockIdx.x * kSvdThreads + threadIdx.x; i < n; i += (long)gridDim.x * kSvdThreads) {
    if (d == 2) {
      float s[2], de[2];
      svd2(J + i * 4, s);
      svd_e<2>(s, ra, rv, de);
      grad2(J + i * 4, go * de[0], go * de[1], gJ + i * 4);
    } else {
      float B[3][3], V[3][3], s[3], de[3];
      const float* Ji = J + i * 9;
      jacobi3(Ji, B, V);
      svd3_sorted(B, V, s);
      svd_e<3>(s, ra, rv, de);
      grad3(Ji, B, V, s, go, de, gJ + i * 9);
    }
  }
}


// ---------------------------------------------------------------------------------------
// The whole elastodynamics energy of one iteration (insr_elastic_energy): one thread per row
// of the trainable field's merged jet; interior rows (< n) carry ARAP / volume (the SVD of
// dq/dx = J + I), kinematics, external force and collision terms, the constraint rows their
// positional terms.  Each term's raw sum is reduced separately (deterministic, block order,
// last block combines), scaled like the reference and added in cfg.energy order; the
// gradient for a unit seed is written in the same pass.
// ---------------------------------------------------------------------------------------
constexpr int kElThreads = 256;
constexpr int kElMaxBlocks = 1024;
// reduced sums: the INSR_EL_TERMS terms' raw sums, then the 3-D sphere's second factor
// (sum qdot . dir over the colliding rows; the term's own slot holds sum |q - c|)
constexpr int kElSphereB = INSR_EL_TERMS;
constexpr int kElAcc = INSR_EL_TERMS + 1;
// work: [kElAcc][kElMaxBlocks] block partials, the ticket, then the 3-D sphere's two sums for
// the gradient pass (elastic_sphere3_grad_kernel)
constexpr long kElTicket = (long)kElAcc * kElMaxBlocks;

__global__ __launch_bounds__(kElThreads) void elastic_energy_kernel(const InsrElastic E, float* __restrict__ work) {
  __shared__ float red[kElAcc][kElThreads / 64];
  const int d = E.d;
  const float dt = E.dt;
  const bool svd = E.ratio[INSR_EL_ARAP] != 0.f || E.ratio[INSR_EL_VOLUME] != 0.f;
  float acc[kElAcc];
#pragma unroll
  for (int t = 0; t < kElAcc; ++t) acc[t] = 0.f;
  for (long r = (long)blockIdx.x * kElThreads + threadIdx.x; r < E.rows; r += (long)gridDim.x * kElThreads) {
    float gf[3] = {0.f, 0.f, 0.f};
    if (r < E.n) {
      float q[3], qd[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        if (k >= d) break;
        const float xk = E.x[r * d + k];
        q[k] = E.f[r * d + k] + xk;                 // q = f(x) + x
        const float qp = E.f_prev[r * d + k] + xk;  // q_prev, q_prev_prev (no grad)
        const float qpp = E.f_pp[r * d + k] + xk;
        qd[k] = (q[k] - qp) / dt;
        if (E.ratio[INSR_EL_KINEMATICS] != 0.f) {  // rk sum (qdot - qdot_prev)^2
          const float a = qd[k] - (qp - qpp) / dt;
          acc[INSR_EL_KINEMATICS] += a * a;
          gf[k] += (E.ratio[INSR_EL_KINEMATICS] * (2.f * a)) / dt;
        }
        if (E.ratio[INSR_EL_EXTERNAL] != 0.f) {  // -dt sum qdot . f_ext
          acc[INSR_EL_EXTERNAL] += qd[k] * E.ext[k];
          gf[k] += (-dt * E.ext[k]) / dt;
        }
      }
      if (E.ratio[INSR_EL_COLLISION] != 0.f) {  // plane: -dt sum qdot_z rc (h - q_z) over q_z < h
        const float qz = q[d - 1];
        if (qz < E.plane_height) {
          const float force = E.ratio[INSR_EL_COLLISION] * (E.plane_height - qz);
          acc[INSR_EL_COLLISION] += qd[d - 1] * force;
          gf[d - 1] += (-dt * force) / dt + dt * qd[d - 1] * E.ratio[INSR_EL_COLLISION];
        }
      }
      if (E.ratio[INSR_EL_SPHERE] != 0.f) {  // sphere: penalty force rc dist dir on rows with dist < R
        float vec[3], ss = 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (k >= d) break;
          vec[k] = q[k] - E.center[k];
          ss += vec[k] * vec[k];
        }
        const float dist = sqrtf(ss);
        if (d == 3) {  // the two factors of the 3-D product; the gradient pass follows the totals
          if (dist < E.radius) {
            acc[INSR_EL_SPHERE] += dist;
            acc[kElSphereB] += qd[0] * (vec[0] / dist) + qd[1] * (vec[1] / dist) + qd[2] * (vec[2] / dist);
          }
        } else if (dist < E.radius) {  // 2-D: -dt sum qdot . rc dist dir
          const float rd = E.ratio[INSR_EL_SPHERE] * dist;
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            if (k >= d) break;
            acc[INSR_EL_SPHERE] += qd[k] * (rd * (vec[k] / dist));
            gf[k] += -E.ratio[INSR_EL_SPHERE] * vec[k] - dt * E.ratio[INSR_EL_SPHERE] * qd[k];
          }
        }
      }
      if (svd) {  // singular values of dq/dx = J + I
        const float ra = E.ratio[INSR_EL_ARAP], rv = E.ratio[INSR_EL_VOLUME];
        if (d == 2) {
          float Jq[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) Jq[k] = E.J[r * 4 + k] + ((k == 0 || k == 3) ? 1.f : 0.f);
          float s[2], de[2];
          svd2(Jq, s);
          svd_e<2>(s, ra, rv, de);
          acc[INSR_EL_ARAP] += (s[0] - 1.f) * (s[0] - 1.f) + (s[1] - 1.f) * (s[1] - 1.f);
          const float pm = s[0] * s[1] - 1.f;
          acc[INSR_EL_VOLUME] += pm * pm;
          if (E.gJ) grad2(Jq, de[0], de[1], E.gJ + r * 4);
        } else {
          float Jq[9];
#pragma unroll
          for (int k = 0; k < 9; ++k) Jq[k] = E.J[r * 9 + k] + ((k % 4 == 0) ? 1.f : 0.f);
          float B[3][3], V[3][3], s[3], de[3];
          jacobi3(Jq, B, V);
          svd3_sorted(B, V, s);
          svd_e<3>(s, ra, rv, de);
          acc[INSR_EL_ARAP] += (s[0] - 1.f) * (s[0] - 1.f) + (s[1] - 1.f) * (s[1] - 1.f) + (s[2] - 1.f) * (s[2] - 1.f);
          const float pm = s[0] * s[1] * s[2] - 1.f;
          acc[INSR_EL_VOLUME] += pm * pm;
          if (E.gJ) grad3(Jq, B, V, s, 1.f, de, E.gJ + r * 9);
        }
      }
    } else {
      if (r >= E.row_l && r < E.row_l + E.n_l) {  // rc sum |f(x_l)|^2
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (k >= d) break;
          const float v = E.f[r * d + k];
          acc[INSR_EL_CONSTRAINT] += v * v;
          gf[k] += E.ratio[INSR_EL_CONSTRAINT] * (2.f * v);
        }
      }
      if (r >= E.row_r && r < E.row_r + E.n_r) {  // rc sum |f(x_r) - target|^2
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (k >= d) break;
          const float v = E.f[r * d + k] - E.target[k];
          acc[INSR_EL_CONSTRAINT_RIGHT] += v * v;
          gf[k] += E.ratio[INSR_EL_CONSTRAINT_RIGHT] * (2.f * v);
        }
      }
      if (E.gJ && svd)
        for (int k = 0; k < d * d; ++k) E.gJ[r * d * d + k] = 0.f;
    }
    if (E.gf)
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (k < d) E.gf[r * d + k] = gf[k];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < kElAcc; ++t) {
    float v = acc[t];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) red[t][w] = v;
  }
  __shared__ float tot[kElAcc];
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x < kElAcc) {  // the block's partial of sum t (waves in order)
    const int t = threadIdx.x;
    float part = 0.f;
#pragma unroll
    for (int k = 0; k < kElThreads / 64; ++k) part += red[t][k];
    tot[t] = part;
    if (gridDim.x > 1)  // sc1 partial store; the wait below covers all eight lanes' stores
      __hip_atomic_store(work + t * kElMaxBlocks + blockIdx.x, part, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) {
    last = 1;
    if (gridDim.x > 1) {  // relaxed ticket after the sc1 stores complete: the hardware hand-off
                          // of block_partial_combine (residual.hip header; no release/acquire)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      unsigned* ticket = reinterpret_cast<unsigned*>(work + kElTicket);
      last = atomicAdd(ticket, 1u) == gridDim.x - 1 ? 1 : 0;
    }
  }
  __syncthreads();
  if (!last) return;
  if (gridDim.x > 1) {
    // the last block: wave w sums w, w + 4, w + 8 over every block's partial, lanes load in
    // parallel (lane l: blocks l, l + 64, ...), fixed butterfly -- deterministic
#pragma unroll
    for (int h = 0; h < (kElAcc + 3) / 4; ++h) {
      const int t = w + 4 * h;
      float v = 0.f;
      if (t < kElAcc)
        for (int q = lane; q < (int)gridDim.x; q += 64)
          v += __hip_atomic_load(work + t * kElMaxBlocks + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      __syncthreads();
      if (lane == 0 && t < kElAcc) tot[t] = v;
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  // scale of each raw sum (the reference's ratio * torch.sum(...), -dt * torch.sum(...)); the
  // total in cfg.energy order (loss = 0; loss = loss + E_t)
  float et[INSR_EL_TERMS];
#pragma unroll
  for (int t = 0; t < INSR_EL_TERMS; ++t) {
    const float scale = (t == INSR_EL_EXTERNAL || t == INSR_EL_COLLISION || t == INSR_EL_SPHERE) ? -dt : E.ratio[t];
    et[t] = scale * tot[t];
    if (t == INSR_EL_SPHERE && d == 3) et[t] = -dt * (E.ratio[t] * tot[t]) * tot[kElSphereB];
    if (E.terms) E.terms[t] = et[t];
  }
  float loss = 0.f;
  for (int k = 0; k < E.n_order; ++k) {
    const int t = E.order[k];
#pragma unroll
    for (int q = 0; q < INSR_EL_TERMS; ++q)
      if (q == t) loss += et[q];
  }
  E.out[0] = loss;
  if (d == 3 && E.ratio[INSR_EL_SPHERE] != 0.f) {  // the two sums, for the gradient pass
    work[kElTicket + 1] = tot[INSR_EL_SPHERE];
    work[kElTicket + 2] = tot[kElSphereB];
  }
  if (gridDim.x > 1) atomicExch(reinterpret_cast<unsigned*>(work + kElTicket), 0u);
}

// The 3-D sphere term's gradient, after elastic_energy_kernel has both sums A = sum |q - c| and
// B = sum qdot . dir (colliding rows): E = -dt rc A B, so on a colliding row
//   dE/dq = -dt rc (B dir + A (dir / dt + (qdot - (qdot . dir) dir) / |q - c|))
// (d|q - c|/dq = dir, d(qdot . dir)/dq = dir / dt + (I - dir dir^T) qdot / |q - c|), added to gf.
__global__ __launch_bounds__(kElThreads) void elastic_sphere3_grad_kernel(const InsrElastic E,
                                                                          const float* __restrict__ work) {
  const float A = work[kElTicket + 1], Bs = work[kElTicket + 2];
  const float dt = E.dt, c = -dt * E.ratio[INSR_EL_SPHERE];
  for (long r = (long)blockIdx.x * kElThreads + threadIdx.x; r < E.n; r += (long)gridDim.x * kElThreads) {
    float vec[3], qd[3], ss = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float xk = E.x[r * 3 + k];
      const float q = E.f[r * 3 + k] + xk;
      qd[k] = (q - (E.f_prev[r * 3 + k] + xk)) / dt;
      vec[k] = q - E.center[k];
      ss += vec[k] * vec[k];
    }
    const float dist = sqrtf(ss);
    if (!(dist < E.radius)) continue;
    float dir[3], qdir = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      dir[k] = vec[k] / dist;
      qdir += qd[k] * dir[k];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k)
      E.gf[r * 3 + k] += c * (Bs * dir[k] + A * (dir[k] / dt + (qd[k] - qdir * dir[k]) / dist));
  }
}

}  // namespace insr

using namespace insr;

extern "C" {

long insr_svd_energy_work_floats(void) { return kSvdMaxBlocks; }

int insr_svd_energy_fwd(const float* J, long n, int d, float ratio_arap, float ratio_volume, float* out, float* work,
                        void* stream) {
  if (!J || !out || n < 0 || (d != 2 && d != 3)) return INSR_EINVAL;
  long nb = (n + 4 * kSvdThreads - 1) / (4 * kSvdThreads);  // ~4 points per thread
  if (nb < 1) nb = 1;
  if (nb > kSvdMaxBlocks) nb = kSvdMaxBlocks;
  if (nb > 1 && !work) return INSR_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(svd_energy_fwd_kernel, dim3((unsigned)nb), dim3(kSvdThreads), 0, st, J, n, d, ratio_arap,
                     ratio_volume, nb > 1 ? work : out);
  if (nb > 1) hipLaunchKernelGGL(svd_combine_kernel, dim3(1), dim3(64), 0, st, work, (int)nb, out);
  return (int)hipGetLastError();
}

int insr_svd_energy_bwd(const float* J, long n, int d, float ratio_arap, float ratio_volume, const float* gout,
                        float* gJ, void* stream) {
  if (!J || !gout || !gJ || n < 0 || (d != 2 && d != 3)) return INSR_EINVAL;
  if (n == 0) return 0;
  long nb = (n + kSvdThreads - 1) / kSvdThreads;
  if (nb > 4096) nb = 4096;
  hipLaunchKernelGGL(svd_energy_bwd_kernel, dim3((unsigned)nb), dim3(kSvdThreads), 0, (hipStream_t)stream, J, n, d,
                     ratio_arap, ratio_volume, gout, gJ);
  return (int)hipGetLastError();
}


long insr_elastic_work_floats(void) { return kElTicket + 4; }

int insr_elastic_energy(const InsrElastic* e, float* work, void* stream) {
  if (!e || (e->d != 2 && e->d != 3) || e->n < 0 || e->rows < e->n || !e->out) return INSR_EINVAL;
  if (e->n > 0 && (!e->f || !e->x || !e->f_prev || !e->f_pp)) return INSR_EINVAL;
  if (e->rows > e->n && !e->f) return INSR_EINVAL;
  const bool svd = e->ratio[INSR_EL_ARAP] != 0.f || e->ratio[INSR_EL_VOLUME] != 0.f;
  if (svd && e->n > 0 && !e->J) return INSR_EINVAL;
  if (!(e->dt > 0.f) || e->n_order < 0 || e->n_order > INSR_EL_TERMS) return INSR_EINVAL;
  const bool sphere3 = e->ratio[INSR_EL_SPHERE] != 0.f && e->d == 3;  // 3-D: a product of two sums
  for (int k = 0; k < e->n_order; ++k)
    if (e->order[k] < 0 || e->order[k] >= INSR_EL_TERMS) return INSR_EINVAL;
  if (e->n_l < 0 || e->n_r < 0 || (e->n_l > 0 && (e->row_l < e->n || e->row_l + e->n_l > e->rows)) ||
      (e->n_r > 0 && (e->row_r < e->n || e->row_r + e->n_r > e->rows)))
    return INSR_EINVAL;
  // one row per thread up to kElMaxBlocks blocks (the per-row chain of dependent loads and the 3x3
  // Jacobi sweeps want parallelism more than per-thread reuse: el2D 14.9 us with 4 rows per thread)
  long nb = (e->rows + kElThreads - 1) / kElThreads;
  if (nb < 1) nb = 1;
  if (nb > kElMaxBlocks) nb = kElMaxBlocks;
  if ((nb > 1 || sphere3) && !work) return INSR_EINVAL;
  hipLaunchKernelGGL(elastic_energy_kernel, dim3((unsigned)nb), dim3(kElThreads), 0, (hipStream_t)stream, *e, work);
  if (sphere3 && e->gf && e->n > 0) {
    long ng = (e->n + kElThreads - 1) / kElThreads;
    if (ng > kElMaxBlocks) ng = kElMaxBlocks;
    hipLaunchKernelGGL(elastic_sphere3_grad_kernel, dim3((unsigned)ng), dim3(kElThreads), 0, (hipStream_t)stream, *e,
                       work);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
