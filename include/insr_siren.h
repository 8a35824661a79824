/*
 * insr_siren.h -- C ABI of libinsr_hip.so, the MI355X (gfx950) hot path of the
 * INSR-PDE per-timestep training loop.
 *
 * The reference (qingxu-thu/INSR-PDE) is pure Python over PyTorch; its "FFI" for
 * this path is the torch dispatcher.  Each entry point below replaces the group
 * of aten kernels the reference's Python launches for one operator:
 *
 *   insr_siren_jet_fwd   MLP.forward (base/networks.py:67-71) + the create_graph
 *                        autograd passes of gradient / divergence / jacobian /
 *                        laplace (base/diff_ops.py:33-82), as ONE forward Taylor
 *                        jet (value, d tangents, Laplacian stream).
 *   insr_siren_jet_bwd   loss.backward() through those graphs down to the
 *                        parameters (base/baseModel.py:77) -- the 2nd/3rd-order
 *                        reverse pass -- as per-block partial gradients.
 *   insr_reduce_partials deterministic sum of the per-block partials into the
 *                        network's flat .grad buffer (autograd's AccumulateGrad).
 *   insr_adam_prepare /  torch.optim.Adam.step() + ReduceLROnPlateau.step()
 *   insr_adam_step       (base/baseModel.py:55-62,79-81) over one flat buffer,
 *                        with lr / step / plateau state kept on the device.
 *
 * Conventions
 *   - Every pointer is a device pointer owned by the caller (torch tensors);
 *     the library never allocates or frees.  Sizes come from the *_bytes /
 *     *_count queries.
 *   - Every call is asynchronous on the caller's hipStream_t (passed as void*);
 *     no host synchronisation, so calls are hipGraph-capturable.
 *   - Return 0 on success, a negative INSR_E* code for a bad argument, or a
 *     positive hipError_t from the launch.  Nothing throws across the ABI.
 *   - Parameters are ONE flat fp32 buffer in torch state_dict order:
 *       net.0.weight (W x d_in), net.0.bias (W),
 *       net.2.weight (W x W), net.2.bias (W), ... (L hidden layers),
 *       net.{2L+2}.weight (d_out x W), net.{2L+2}.bias (d_out)
 *     i.e. nn.Linear's (out, in) row-major weights, exactly as the reference
 *     stores them (base/networks.py:50-60), so state_dicts load unchanged.
 */
#ifndef INSR_SIREN_H
#define INSR_SIREN_H

#ifdef __cplusplus
extern "C" {
#endif

/* jet modes: which derivative streams ride along with the value */
#define INSR_MODE_VALUE 0 /* y                                  (1 stream)        */
#define INSR_MODE_GRAD  1 /* y, dy/dx_i  (Jacobian rows)         (1 + d_in streams) */
#define INSR_MODE_LAP   2 /* y, dy/dx_i, sum_i d2y/dx_i^2        (2 + d_in streams) */
#define INSR_MODE_MASK  0xF
/* Per-call matrix-core precision: OR INSR_JET_PREC(p) (p an INSR_PREC_* below) into the
 * `mode` argument of any jet entry point or query; without it the default (f16x3 forward,
 * bf16x6 backward) applies.  The saved-activation layout does not depend on it. */
#define INSR_MODE_PREC_SHIFT 4
#define INSR_JET_PREC(p) (((p) + 1) << INSR_MODE_PREC_SHIFT)
/* Backward-only override (a "mixed" precision: e.g. a bf16x3 forward with a bf16 backward):
 * OR INSR_JET_BPREC(p) as well; the backward of the call then runs at p, the forward at the
 * INSR_JET_PREC / process-default precision. */
#define INSR_MODE_BPREC_SHIFT 12
#define INSR_JET_BPREC(p) (((p) + 1) << INSR_MODE_BPREC_SHIFT)
/* INSR_MODE_WSPLIT: the params buffer carries the pre-split weight planes of
 * insr_siren_wsplit() after the parameters (at insr_siren_wsplit_offset() floats), up to date
 * with the parameters.  Without it an entry point that runs split-bf16 kernels splits the
 * weights itself, into a per-stream scratch copy (one copy + one launch per call). */
#define INSR_MODE_WSPLIT (1 << 8)
/* Per-call knobs (A/B studies; every field 0 = the library's measured policy).  The library keeps
 * no mutable process-wide configuration and reads no environment: calls on distinct streams or
 * host threads with different knobs are independent (re-entrant).  OR them into `mode` of the
 * jet entry points and of the host queries (insr_jet_bwd_path, *_work_bytes, ...); a forward and
 * the backward of its saved streams must carry the same knobs.
 *   INSR_JET_POLICY(p)     backward path: 0 auto, 1 fused tile-split where it exists, 2 two-kernel,
 *                          3 resident dW (bf16x6 kernel), 4 recompute where it applies, 5 resident dW
 *                          with f16x3 products (the saved-stream variant of the recompute kernel;
 *                          auto for 2-d Laplacian jets from 4,096 points) (insr_jet_bwd_path)
 *   INSR_JET_BWD_F16(m)    mask of INSR_BWD_F16_* products of the x6 backward on the fp16 matrix
 *                          cores (0..7; without the field: all three)
 *   INSR_JET_TILES(f,b,m)  tile-split blocks: forced forward / backward tiles per block (0 auto,
 *                          1, 2, 4: the largest feasible T not above) and the minimum block count
 *                          of the auto choice (INSR_MINB_256 (default) / _512 / _128 / _1024)
 *   INSR_MODE_WIDE128      the two-kernel backward from width 128 (else from 256, plus the
 *                          measured width-128 batch thresholds) */
#define INSR_MODE_WIDE128 (1 << 9)
#define INSR_MODE_POLICY_SHIFT 16
#define INSR_JET_POLICY(p) (((p) + 1) << INSR_MODE_POLICY_SHIFT)
#define INSR_MODE_F16_SHIFT 19
#define INSR_JET_BWD_F16(m) (((m) + 1) << INSR_MODE_F16_SHIFT)
#define INSR_MODE_TILES_SHIFT 23
#define INSR_TILES_CODE(t) ((t) == 4 ? 3 : ((t) == 2 ? 2 : ((t) == 1 ? 1 : 0)))
#define INSR_MINB_256 0
#define INSR_MINB_512 1
#define INSR_MINB_128 2
#define INSR_MINB_1024 3
#define INSR_JET_TILES(f, b, minb) \
  ((INSR_TILES_CODE(f) | (INSR_TILES_CODE(b) << 2) | ((minb) << 4)) << INSR_MODE_TILES_SHIFT)

#define INSR_EINVAL   (-1) /* unsupported shape / mode / null pointer */
#define INSR_EWIDTH   (-2) /* hidden width not in the compiled set      */
#define INSR_ENOCOMM  (-3) /* RCCL (librccl.so.1) could not be loaded   */
#define INSR_ECAPTURE (-4) /* a per-stream scratch would be allocated during stream capture:
                              run the call once outside the capture, or pass INSR_MODE_WSPLIT */
#define INSR_ERANGE   (-5) /* a hidden weight |w| >= 255 reached the fp16 weight planes (insr_siren_wsplit_status) */
#define INSR_ECOMM_BASE 1000 /* + ncclResult_t of a failed RCCL call     */

/* Library version (major*10000 + minor*100 + patch). */
int insr_version(void);

/* Build provenance: the first 16 hex digits of the SHA-256 of the sources the library was
 * built from (the csrc .hip and .hpp files in name order, then this header). */
const char* insr_build_id(void);

/* Number of fp32 parameters of an SIREN(d_in -> W x (L+1) -> d_out). */
long insr_siren_param_count(int d_in, int d_out, int num_hidden, int width);

/* Pre-split weight planes (split-bf16 kernels).  Every hidden weight W_j is stored split in
 * three bf16 terms (jet_x6.hpp) in the matrix-core fragment order of the forward (W_j rows)
 * and of the backward (W_j^T rows), then 2^8 W_j split in two fp16 terms in the forward and in
 * the backward order (INSR_PREC_F16X3): 5 L W^2 floats, then a status quad (4 floats) -- in all
 * insr_siren_wsplit_floats(), at insr_siren_wsplit_offset() floats (param_count rounded up to 16 B)
 * after the start of the params buffer.
 * insr_siren_wsplit() writes them from the parameters in place (one launch); the kernels then
 * read fragments instead of re-splitting W in every block.  Replaces nothing in the
 * reference (its fp32 addmm reads W directly, torch/nn/modules/linear.py). */
long insr_siren_wsplit_offset(int d_in, int d_out, int num_hidden, int width);
long insr_siren_wsplit_floats(int num_hidden, int width);
int insr_siren_wsplit(float* params, int d_in, int d_out, int num_hidden, int width, void* stream);
/* Range guard of the fp16 planes: 2^8 w in fp16 needs |w| < 255.  insr_siren_wsplit and the Adam launches
 * that keep the planes current (insr_adam_step_nets / insr_adam_plateau_step_nets with shapes) flag any
 * hidden weight outside that range in the status quad (and clamp its fp16 terms, so nothing overflows;
 * the f16x3 products of that layer are then not the network's -- the bf16 planes, fp32's range, are
 * exact).  Returns INSR_ERANGE when flagged, 0 when not (waits for `stream`; a host sync point).
 * insr_siren_wsplit clears the flag; the Adam launches only set it. */
int insr_siren_wsplit_status(const float* params, int d_in, int d_out, int num_hidden, int width, void* stream);

/* 1 if (d_in, d_out, width, mode) is served by a compiled kernel, else 0. */
int insr_siren_supported(int d_in, int d_out, int num_hidden, int width, int mode);

/* Bytes of the activation buffer the forward saves for the backward. */
long insr_jet_act_bytes(long n_points, int d_in, int num_hidden, int width, int mode);

/* Bytes of the per-block partial-gradient buffer the backward writes. */
long insr_jet_partial_bytes(long n_points, int d_in, int d_out, int num_hidden, int width, int mode);

/*
 * Forward jet over n_points collocation points.
 *   x    (n, d_in)                      sample coordinates
 *   y    (n, d_out)                     network value
 *   dy   (n, d_out, d_in)  [GRAD, LAP]  Jacobian d y_o / d x_i (else may be NULL)
 *   lap  (n, d_out)        [LAP]        sum_i d2 y_o / dx_i^2   (else may be NULL)
 *   act  insr_jet_act_bytes            saved pre-activation streams for
 *                                       insr_siren_jet_bwd; NULL = inference only.
 * Replaces: base/networks.py:67-71 and base/diff_ops.py:33-82.
 */
int insr_siren_jet_fwd(const float* x, long n_points, int d_in, int d_out, int num_hidden,
                       int width, int mode, const float* params, float* y, float* dy, float* lap,
                       float* act, void* stream);

/*
 * Several independent forward jets of ONE architecture and mode in one launch
 * (horizontal fusion): each job is an insr_siren_jet_fwd call's own buffers
 * (its network's params, its points). Results are those of insr_siren_jet_fwd
 * per job, bit for bit, and each job's act feeds insr_siren_jet_bwd as usual.
 * Used where a model phase evaluates two networks (or one network at two
 * batches) with no dependency between them, e.g. the frozen and the trainable
 * velocity fields at the same collocation points (fluid/model.py:97-98 and
 * :143-147): a value jet of 16384 points is a latency-bound launch that holds
 * one block per CU, so two side by side cost well under two launches.
 * 1 <= n_jobs <= INSR_MAX_FWD_JOBS; jobs with n == 0 are allowed. The output width
 * may differ per job (InsrJetJob.d_out: e.g. the velocity and pressure fields).
 * Replaces: consecutive MLP.forward calls (base/networks.py:67-71).
 */
#define INSR_MAX_FWD_JOBS 6
typedef struct InsrJetJob {
  const float* x;       /* (n, d_in) */
  const float* params;  /* flat parameters of this job's network */
  float* y;             /* (n, d_out) */
  float* dy;            /* (n, d_out, d_in) [GRAD, LAP] else NULL */
  float* lap;           /* (n, d_out) [LAP] else NULL */
  float* act;           /* insr_jet_act_bytes(n, ...) or NULL (no backward) */
  long n;               /* points of this job */
  int d_out;            /* this job's output width (1..3); 0 = the call's d_out */
} InsrJetJob;
/* Independent forward jets of one width / d_in / depth with DIFFERENT jet modes in one launch
 * (modes[k] = INSR_MODE_VALUE / GRAD / LAP of job k; prec_mode = the common precision and
 * INSR_MODE_WSPLIT bits, no jet-mode bits).  Each job's outputs and saved streams equal its
 * own insr_siren_jet_fwd call bit for bit (its own body and tile count; one launch at
 * W = 128 split-bf16, one launch per job otherwise).  Replaces: consecutive MLP.forward +
 * diff-op calls of a phase (fluid/model.py:106-111, :143-147). */
/* modes[k] = INSR_MIX_ADVECT: the semi-Lagrangian target of the fluid advection
 * (fluid/model.py:96-97) in one job: y = f(clamp(x - dt f(x), lo, hi)) with the job's
 * network f (value jets, d_out == d_in), f(x) written to the job's dy field (n, d_out) and
 * the foot to its lap field (n, d_in); scalars[3 k .. 3 k + 2] = (dt, lo, hi). */
#define INSR_MIX_ADVECT 3
int insr_siren_jet_fwd_mixed(const InsrJetJob* jobs, const int* modes, const float* scalars, int n_jobs, int d_in,
                             int d_out, int num_hidden, int width, int prec_mode, void* stream);
int insr_siren_jet_fwd_multi(const InsrJetJob* jobs, int n_jobs, int d_in, int d_out,
                             int num_hidden, int width, int mode, void* stream);

/*
 * Backward of the jet to the parameters.  Adjoints (any may be NULL = zero):
 *   gy (n, d_out), gdy (n, d_out, d_in), glap (n, d_out).
 *   partial  insr_jet_partial_bytes: one fp32 parameter-gradient row per block
 *            (insr_jet_partial_blocks(n, d_in, width, mode) rows of
 *            insr_jet_partial_stride(...) floats; the first param_count are used).
 * Sum the rows with insr_reduce_partials_strided into the network's flat .grad.
 * The gradient w.r.t. x is not produced (the reference never reads it).
 * Replaces: the autograd backward of loss.backward() (base/baseModel.py:77).
 */
int insr_siren_jet_bwd(const float* x, long n_points, int d_in, int d_out, int num_hidden,
                       int width, int mode, const float* params, const float* act,
                       const float* gy, const float* gdy, const float* glap, float* partial,
                       void* stream);

/*
 * Backward of the jet straight into the network's flat gradient (act may be NULL when
 * insr_jet_bwd_path() is 3: the recompute backward reads only x, the params and the adjoints):
 *   grad = (accumulate ? grad : 0) + d(loss)/d(params)   (fixed summation order)
 *   work  insr_jet_bwd_work_bytes(...) of scratch.
 * Width <= 128 (and F32 backward precision): insr_siren_jet_bwd + insr_reduce_partials.
 * Width 256 with the x6 backward precision: the wide path (jet_x6w.hip) -- a
 * propagation-only reverse sweep storing the pre-activation adjoints, a split-K GEMM
 * for the hidden-layer weight gradients (K = points x streams), compact partial rows
 * for the first layer, the biases and the output layer, and their reductions.
 * Replaces: loss.backward() into the parameters (base/baseModel.py:77).
 */
int insr_siren_jet_bwd_grad(const float* x, long n_points, int d_in, int d_out, int num_hidden,
                            int width, int mode, const float* params, const float* act,
                            const float* gy, const float* gdy, const float* glap, float* work,
                            float* grad, int accumulate, void* stream);
long insr_jet_bwd_work_bytes(long n_points, int d_in, int d_out, int num_hidden, int width, int mode);

/*
 * Several backward jobs of ONE network and jet mode -- the network's forward jets of one
 * loss.backward(), e.g. a phase's interior batch and its boundary bands evaluated by
 * separate network calls (fluid/model.py:80,96-97: curr_u, vel_x, vel_y) -- straight into
 * its flat gradient:  grad = (accumulate ? grad : 0) + sum_k d(loss)/d(params) of job k.
 * Jobs the fused tile-split backward serves share ONE launch (blocks [first[k], first[k+1])
 * run job k; a 162-point band adds its tiles to the interior's launch instead of a
 * latency-bound launch of its own) and ONE fixed-order reduction of all their partial rows;
 * a job another path serves at its size (two-kernel, resident) runs as its own
 * insr_siren_jet_bwd_grad.  work: insr_jet_bwd_multi_work_bytes(...) of scratch.
 * 1 <= n_jobs <= INSR_MAX_BWD_JOBS; jobs with n == 0 are skipped.
 * Replaces: the per-call autograd backwards of loss.backward() (base/baseModel.py:77).
 */
#define INSR_MAX_BWD_JOBS 8
typedef struct InsrBwdJob {
  const float* x;     /* (n, d_in) points of the forward */
  const float* act;   /* the forward's saved streams (insr_jet_act_bytes(n, ...)) */
  const float* gy;    /* (n, d_out) or NULL */
  const float* gdy;   /* (n, d_out, d_in) or NULL */
  const float* glap;  /* (n, d_out) or NULL */
  long n;
} InsrBwdJob;
int insr_siren_jet_bwd_grad_multi(const InsrBwdJob* jobs, int n_jobs, int d_in, int d_out, int num_hidden,
                                  int width, int mode, const float* params, float* work, float* grad,
                                  int accumulate, void* stream);
/* Scratch bytes of insr_siren_jet_bwd_grad_multi for jobs of n[0..n_jobs) points. */
long insr_jet_bwd_multi_work_bytes(const long* n, int n_jobs, int d_in, int d_out, int num_hidden, int width,
                                   int mode);
/* The reverse jets of insr_siren_jet_bwd_grad_multi WITHOUT their sums, when every job takes the fused
 * tile-split path: one launch writes the jobs' partial-gradient rows into `work` (row stride
 * insr_jet_partial_stride) and the call returns the number of rows (>= 0); the caller sums them later --
 * insr_reduce_partials_strided, or insr_adam_step_partials (the sums with the Adam update, one launch: the
 * reference's separate interior / band calls of one network, fluid/model.py:80,96-97, then cost what one
 * merged call costs).  INSR_EINVAL when a job takes another path (use insr_siren_jet_bwd_grad_multi). */
int insr_siren_jet_bwd_multi_rows(const InsrBwdJob* jobs, int n_jobs, int d_in, int d_out, int num_hidden,
                                  int width, int mode, const float* params, float* work, void* stream);
/* The reverse jets of several calls of ONE network (the reference's interior + band calls of a Laplacian
 * loss, fluid/model.py:111,119-120) as ONE launch of the saved-stream resident sweep (jet_fb.hpp) when that
 * sweep serves the jobs' total point count, or (round 6) as ONE propagation + ONE split-K dW launch of the
 * two-kernel backward (jet_x6w.hpp) when that path serves 16 * (total 16-point tiles) points (the reference's
 * elasticity interior + constraint calls, elasticity/model.py:137,161-174): phase 1 of
 * insr_siren_jet_bwd_grad_adam for all jobs at once.  The partials land in `work`
 * (insr_jet_bwd_work_bytes(16 * total tiles, ...)); phase 2 -- insr_siren_jet_bwd_grad_adam(..., n_points =
 * 16 * (total 16-point tiles), phases = 2, ...), with or without the Adam update -- sums them.  INSR_EINVAL
 * when another path serves that total. */
int insr_siren_jet_bwd_multi_sweep(const InsrBwdJob* jobs, int n_jobs, int d_in, int d_out, int num_hidden,
                                   int width, int mode, const float* params, float* work, void* stream);
/* 1 if insr_siren_jet_bwd_grad takes the wide path for this batch / width / mode. */
int insr_jet_bwd_is_wide(long n_points, int d_in, int width, int mode);

/* Which backward serves this jet: 0 = the fused tile-split kernel writing partial rows
 * (insr_siren_jet_bwd + insr_reduce_partials_strided), 1 = the two-kernel path, 2 = the
 * resident-dW persistent kernel (W = 128, <= 4 hidden layers: every hidden layer's weight
 * gradient held in registers across the batch, the saved streams read once, no adjoint round
 * trip through memory; f16x3 products with per-tile scales for 4-hidden-layer nets while the
 * INSR_BWD_F16_FUSED bit is on -- the 2-d Laplacian jets from 4,096 points by default -- else
 * bf16x6), 3 = the RECOMPUTE backward (W = 128, 4 hidden
 * layers, fp32-level backward precision: one persistent launch that reruns the forward jet of
 * each 16-point tile next to its reverse jet, dW resident per CU -- it reads no saved streams,
 * so the forward of such a call passes act = NULL and saves nothing).  1, 2 and 3 run through
 * insr_siren_jet_bwd_grad with an insr_jet_bwd_work_bytes workspace; path 3 never depends on
 * n_points (the forward's decision and the backward's agree). */
int insr_jet_bwd_path(long n_points, int d_in, int d_out, int num_hidden, int width, int mode);
/* Which kernel family serves the path above: 1 = jet_fb_x6 (the recompute kernel, path 3, or its
 * saved-stream variant on path 2: f16x3 products), 0 = the path's other kernels (profilers, bench.py). */
int insr_jet_bwd_kernel(long n_points, int d_in, int d_out, int num_hidden, int width, int mode);

/* Matrix products of the x6 (fp32-level) backward that run on the fp16 matrix cores instead of
 * six bf16 products: f16x3 (two fp16 terms per operand, three products, 22 significant bits),
 * the adjoints scaled by the power of two that maps the largest |value| of their K slice / tile
 * into [2^14, 2^15) (undone exactly), the weights by 2^8 (the fp16 planes).  Bits of the per-call
 * INSR_JET_BWD_F16 mask (default: all three):
 * INSR_BWD_F16_DW the two-kernel path's dW GEMM, INSR_BWD_F16_PROP its adjoint propagation,
 * INSR_BWD_F16_FUSED the fused tile-split kernel. */
#define INSR_BWD_F16_DW 1
#define INSR_BWD_F16_PROP 2
#define INSR_BWD_F16_FUSED 4 /* the fused tile-split backward (dW and propagation, per-block scales) */
/* Threads of the three launches of a two-kernel backward (propagation, dW partials, dW sums),
 * as profilers report them; INSR_EINVAL when (n, shape, mode) does not take that path. */
int insr_jet_wide_launch_threads(long n_points, int d_in, int d_out, int num_hidden, int width, int mode,
                                 long* threads3);
/* Number of partial-gradient rows insr_siren_jet_bwd writes for n points: one per
 * T-tile (16T-point) block, T as the backward selects for this size, width and mode. */
int insr_jet_partial_blocks(long n_points, int d_in, int width, int mode);

/* Tiles per tile-split block (1, 2 or 4) the forward (backward != 0: the
 * backward) uses for this batch. */
int insr_jet_split_tiles(long n_points, int d_in, int width, int mode, int backward);

/*
 * Matrix-core precision of the hidden-layer GEMMs (per call: INSR_JET_PREC(p) / INSR_JET_BPREC(p)
 * in its mode; the defaults are f16x3 forward, bf16x6 backward):
 *   INSR_PREC_F32     v_mfma_f32_16x16x4_f32: exact fp32 products, the fp32 matrix rate.
 *   INSR_PREC_BF16X6  every fp32 operand split in three bf16 terms, six
 *                     v_mfma_f32_16x16x32_bf16 products per K chunk, fp32 accumulation:
 *                     fp32-level accuracy (dropped terms <= 2^-26 |a||b|) at 2.67x
 *                     the fp32 matrix throughput.  The default backward.
 *   INSR_PREC_BF16X3  two bf16 terms per operand, three products (dropped terms
 *                     <= 2^-16 |a||b|): 5.3x the fp32 matrix rate.
 *   INSR_PREC_BF16    plain bf16 operands, one product, fp32 accumulation: 16x.
 *   INSR_PREC_F16X3   FORWARD ONLY: every operand scaled by a power of two and split in two
 *                     fp16 terms (11 + 11 significant bits), three v_mfma_f32_16x16x32_f16 products
 *                     per K chunk (dropped term <= 2^-22 |a||b|): fp32-level accuracy at 5.3x the
 *                     fp32 matrix rate.  The default forward.  A backward asked for at this
 *                     precision runs BF16X6.  Scales: the weights x 2^8 (the fp16 planes); the
 *                     Laplacian stream per tile by the power of two that maps its block maximum
 *                     into [2^14, 2^15); the tangent streams unscaled while their bound w |t| stays
 *                     below 2^15, else (a uniform branch, rare) by their own block power of two; all
 *                     undone exactly on the products.  Range: |W| < 255 (the weight planes), the
 *                     streams fp32's.  The f16 backward products (INSR_JET_BWD_F16, the
 *                     recompute path) scale their adjoints and h operands the same way.
 * The first (K = d_in) and output (M = d_out) layers and every sine stay fp32.
 * The saved-activation and partial
 * layouts do not depend on it: a forward of one precision pairs with a backward of
 * another.
 */
#define INSR_PREC_F32    0
#define INSR_PREC_BF16X6 1
#define INSR_PREC_BF16X3 2
#define INSR_PREC_BF16   3
#define INSR_PREC_F16X3  4

/* grad[i] = (accumulate ? grad[i] : 0) + sum_b partial[b * count + i], fixed order. */
int insr_reduce_partials(const float* partial, int n_blocks, long count, float* grad,
                         int accumulate, void* stream);
/* Row stride (floats) of insr_siren_jet_bwd's partial rows: param_count rounded up to a
 * multiple of 4 (16-B aligned rows; the padding is never read). */
long insr_jet_partial_stride(int d_in, int d_out, int num_hidden, int width);
/* grad[i] = (accumulate ? grad[i] : 0) + sum_b partial[b * stride + i], i < count, fixed
 * order; 16-B loads when stride % 4 == 0 and partial is 16-B aligned.  Many rows are
 * summed in two levels IN PLACE: `partial` is scratch (its rows are overwritten). */
int insr_reduce_partials_strided(const float* partial, int n_blocks, long count, long stride,
                                 float* grad, int accumulate, void* stream);

/*
 * Device-resident optimiser state (INSR_OPT_NFLOATS floats, caller-allocated):
 *   [0] lr  [1] step t  [2] plateau best  [3] plateau num_bad
 *   [4] step_size = lr / (1 - b1^t)        [5] sqrt(1 - b2^t)
 *   [6] plateau factor  [7] plateau min_lr
 * Keeping these on the device lets one training iteration be replayed from a
 * hipGraph with no host round trip (the reference syncs twice per iteration,
 * base/baseModel.py:81,116).
 */
#define INSR_OPT_LR 0
#define INSR_OPT_STEP 1
#define INSR_OPT_BEST 2
#define INSR_OPT_BAD 3
#define INSR_OPT_STEPSIZE 4
#define INSR_OPT_BC2SQRT 5
#define INSR_OPT_FACTOR 6
#define INSR_OPT_MINLR 7
#define INSR_OPT_TICKET 8 /* (as unsigned) insr_adam_plateau_step_nets' last-block ticket, 0 */
#define INSR_OPT_TICKET_SHARDS 9 /* [9, 17): its 8 first-level shards (as unsigned), 0 */
#define INSR_OPT_NFLOATS 17

/* t += 1; refresh step_size and sqrt(1-b2^t) (explicit-prepare convention). */
int insr_adam_prepare(float* opt_state, float beta1, float beta2, void* stream);

/* One ReduceLROnPlateau.step(*loss) (mode min, rel threshold 1e-4, cooldown 0,
 * eps 1e-8), base/baseModel.py:61-62,80-81.  advance_step != 0 also does t += 1
 * (the fused-Adam convention: the update of iteration t used st[STEP] + 1).
 * loss == NULL with advance_step != 0 only advances t. */
int insr_plateau_step(float* opt_state, const float* loss, int patience, int advance_step, void* stream);

/* Adam over up to INSR_ADAM_MAX_TENSORS flat buffers in ONE launch (torch op order).
 * Bias corrections use t = opt_state[STEP] + step_offset. */
#define INSR_ADAM_MAX_TENSORS 8
/* insr_adam_step_multi plus, per buffer, shapes[4 k .. 4 k + 3] = (d_in, d_out, num_hidden,
 * width) of a SIREN flat params buffer (param_count floats) that carries pre-split weight
 * planes (INSR_MODE_WSPLIT): the launch rewrites the planes of every updated hidden weight as
 * well (all zeros / shapes == NULL: a plain buffer). */
int insr_adam_step_nets(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                        float* const* exp_avg_sq, const long* sizes, const int* shapes, const float* opt_state,
                        float beta1, float beta2, float eps, int step_offset, void* stream);
/* insr_adam_step_nets (step_offset 1) followed by insr_plateau_step(opt_state, loss, patience,
 * advance_step = 1) in the SAME launch: the last block to finish runs the scheduler step after
 * every block has read the lr it updates -- a two-level agent-scope ticket (block b adds to shard
 * b % 8, the last adder of a shard to opt_state[INSR_OPT_TICKET]; the last of those resets all
 * nine words), so no word takes more than ~1/8 of the blocks' atomics.
 * base/baseModel.py:79-81 (optimizer.step(); scheduler.step(loss)). */
int insr_adam_plateau_step_nets(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                                float* const* exp_avg_sq, const long* sizes, const int* shapes, float* opt_state,
                                float beta1, float beta2, float eps, const float* loss, int patience, void* stream);
/* insr_siren_jet_bwd_grad in two halves for the backwards the jet_fb.hpp kernel serves (the recompute
 * path and the resident sweep on the saved streams, insr_jet_bwd_kernel == 1) and for the two-kernel
 * path (insr_jet_bwd_path == 1, num_hidden > 0); else INSR_EINVAL:
 * phases 1 = the reverse sweep into `work`, 2 = the sums of `work` into grad, 3 = both.  With
 * exp_avg != NULL the sums run the Adam update of every element they write (t = opt_state[STEP] + 1,
 * the weight planes too under INSR_MODE_WSPLIT) and, loss != NULL, the plateau step after the last
 * block -- insr_siren_jet_bwd_grad + insr_adam_plateau_step_nets in one launch fewer; the same sums
 * and update, bit for bit.  params is read by phase 1 and updated by phase 2. */
int insr_siren_jet_bwd_grad_adam(const float* x, long n_points, int d_in, int d_out, int num_hidden, int width,
                                 int mode, float* params, const float* act, const float* gy, const float* gdy,
                                 const float* glap, float* work, float* grad, int accumulate, int phases,
                                 float* exp_avg, float* exp_avg_sq, float* opt_state, float beta1, float beta2,
                                 float eps, const float* loss, int patience, void* stream);
/* The partial-gradient rows of a fused-path backward (insr_siren_jet_bwd's `partial`: nb rows of
 * `stride` floats, insr_jet_partial_blocks / insr_jet_partial_stride) summed into grad (+= with
 * accumulate) -- the same sums, bit for bit, as insr_reduce_partials_strided -- with the Adam update
 * of those count elements (t = opt_state[STEP] + 1; shape as insr_adam_step_nets: the weight planes
 * too) in the same launch, and with loss != NULL the plateau step after the last block
 * (insr_adam_plateau_step_nets' ticket).  One launch instead of the sums + the Adam launch, for a
 * flat buffer whose whole gradient is that backward's.  nb < 1024 (the one-level sums), stride a
 * multiple of 4, partial 16-B aligned; else INSR_EINVAL. */
int insr_adam_step_partials(const float* partial, int nb, long stride, float* grad, int accumulate, float* params,
                            float* exp_avg, float* exp_avg_sq, long count, const int* shape, float* opt_state,
                            float beta1, float beta2, float eps, const float* loss, int patience, void* stream);
int insr_adam_step_multi(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                         float* const* exp_avg_sq, const long* sizes, const float* opt_state, float beta1,
                         float beta2, float eps, int step_offset, void* stream);

/* Single-buffer Adam, explicit-prepare convention (t = opt_state[STEP]). */
int insr_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                   long count, const float* opt_state, float beta1, float beta2, float eps,
                   void* stream);

/*
 * Fused squared-residual losses (the reductions that close every phase's PDE
 * residual: fluid/model.py:96-101,121-125,147-151, the wall terms :90-94,129-133,
 * advection/model.py:78-91).  One launch forward, one backward.
 *   INSR_LOSS_COMBO  out = scale * sum_{i<n} r_i^2,
 *                    r = alpha (a + beta b) + gamma (c + delta d), evaluated in that
 *                    order; b, c, d may be NULL (= 0; d needs c); all contiguous, n elements
 *   INSR_LOSS_BANDS  out = scale * (sum_{r<n} y[r][0]^2 + sum_{r<n} y[n+r][1]^2)
 *                    (a = y, (2n, m) row-major, m >= 2; c = d = NULL), or, with b != NULL,
 *                    scale * (sum_{r<n} a[r][0]^2 + sum_{r<n} b[r][1]^2): the two bands in
 *                    tensors of their own ((n, m) each, the reference's separate band calls
 *                    fluid/model.py:96-98,119-122)
 * The forward reduction is deterministic (fixed order).  Up to 4096 terms it is one
 * launch; beyond, per-block partials go to `work` (insr_sq_loss_work_floats()
 * floats, ZERO-initialised once by the caller, not shared by concurrent launches)
 * and the last block to finish combines them in block order (same launch; it
 * leaves the work's ticket word zero again).
 * Backward: g = 2 scale gout r;  ga = alpha g, gb = alpha beta g, gc = gamma g,
 * gd = gamma delta g (bands: ga = the full (2n, m) gradient, zeros outside the
 * selected columns; with b: ga and gb the full (n, m) gradients of a and b); any output may be
 * NULL (bands: at least one).
 */
#define INSR_LOSS_COMBO 0
#define INSR_LOSS_BANDS 1
long insr_sq_loss_work_floats(void);
int insr_sq_loss_fwd(int kind, const float* a, const float* b, const float* c, const float* d, long n, int m,
                     float alpha, float beta, float gamma, float delta, float scale, float* out, float* work,
                     void* stream);
/* A group of up to INSR_LOSS_GROUP_MAX losses (every residual term of one phase iteration)
 * in ONE launch, each with its gradient for a unit output seed (the training loop's backward
 * seeds every loss with 1): loss k = insr_sq_loss_fwd of (kind, a..d, n, m, coefficients,
 * scale) written to *out, and d(out)/d(input) to ga / gb / gc / gd (any may be NULL).
 * The loss reads a from element a_off (COMBO: n terms; BANDS: rows a_off / m .. a_off / m + 2n
 * of an (R, m) tensor, a_off a multiple of m), b, c, d from element 0 with element strides
 * sb, sc, sd (e.g. the diagonal of a Jacobian).  ga is written on elements [ga_lo, ga_hi):
 * the loss's terms, zeros elsewhere in that range -- two losses over disjoint rows of ONE
 * tensor (a merged jet's interior and band rows) share one gradient buffer; gb / gc / gd are
 * n contiguous elements (gb_len ... = n, or 0 when NULL; BANDS with b: gb = b's n x m gradient).  work: insr_sq_loss_work_floats()
 * floats, zero-initialised once (left zero).  A unit-seeded loss's backward then needs no
 * launch. */
/* out[i] = clamp(x[i] + alpha y[i], lo, hi), i < n: the semi-Lagrangian foot of the fluid
 * advection, clamp(x - dt u_prev(x), -1, 1) (fluid/model.py:97), in one launch. */
int insr_axpy_clamp(const float* x, const float* y, float alpha, float lo, float hi, float* out, long n,
                    void* stream);

#define INSR_LOSS_GROUP_MAX 4
typedef struct InsrLoss {
  int kind;  /* INSR_LOSS_COMBO / INSR_LOSS_BANDS */
  int m;     /* BANDS: columns of a */
  long n;    /* COMBO: terms; BANDS: rows per band */
  const float *a, *b, *c, *d;
  long sb, sc, sd; /* element strides of b, c, d */
  float alpha, beta, gamma, delta, scale;
  float* out;
  float* ga;
  long ga_lo, ga_hi, a_off;
  float *gb, *gc, *gd;
  long gb_len, gc_len, gd_len;
} InsrLoss;
int insr_sq_loss_group(const InsrLoss* losses, int count, float* work, void* stream);
int insr_sq_loss_bwd(int kind, const float* a, const float* b, const float* c, const float* d, long n, int m,
                     float alpha, float beta, float gamma, float delta, float scale, const float* gout, float* ga,
                     float* gb, float* gc, float* gd, void* stream);

/*
 * Adjoint seeds formed inside the reverse jet (round 5).  The unit-seeded gradient of a loss group
 * (insr_sq_loss_group) with respect to a jet's own output is point-local -- 2 scale alpha r at a
 * COMBO term, 2 scale y at a selected BANDS element -- so the backward that consumes it can evaluate
 * it where it reads its adjoint, and emit the squares of the terms its blocks seed: the group's
 * launch disappears from the iteration (base/baseModel.py:73-78 seeds every loss with 1;
 * fluid/model.py:96-101,121-125,147-151 and the wall terms are such groups).  A term seeds the
 * elements [a_off, a_off + n) (COMBO) / the selected elements of rows a_off / m .. + 2n (BANDS) of
 * ONE adjoint stream of the jet -- `a` is that stream's output buffer (y, dy or lap), read at the
 * same elements as insr_sq_loss_group reads them; b, c, d, the coefficients and scale as InsrLoss.
 * The seeds are bit for bit the gradient insr_sq_loss_group writes; each block of the launch writes
 * its terms' square sums to loss_part[block][INSR_SEED_MAX] (term `loss` into column `loss`, other
 * columns 0), and the sums launch that follows the backward finishes the loss values (InsrLossFin:
 * out[k] = scale[k] * sum over the rows of column k, a fixed order; with an Adam + plateau epilogue,
 * before the plateau step reads out[0]).
 */
#define INSR_SEED_MAX 4
#define INSR_SEED_VALUE 0 /* the adjoint of y (gy) */
#define INSR_SEED_GRAD 1  /* of dy (gdy) */
#define INSR_SEED_LAP 2   /* of lap (glap) */
typedef struct InsrSeed {
  int kind;   /* INSR_LOSS_COMBO / INSR_LOSS_BANDS */
  int m;      /* BANDS: columns of a */
  int stream; /* INSR_SEED_VALUE / _GRAD / _LAP */
  int loss;   /* column 0 .. INSR_SEED_MAX - 1 of loss_part */
  long n, a_off;
  const float *a, *b, *c, *d;
  long sb, sc, sd;
  float alpha, beta, gamma, delta, scale;
} InsrSeed;
typedef struct InsrLossFin {
  const float* part; /* loss_part of the seeded backward */
  int rows;          /* its rows (insr_jet_bwd_seed_rows) */
  int nloss;         /* columns 0 .. nloss - 1 -> out[0 .. nloss - 1] */
  float scale[INSR_SEED_MAX];
  float* out[INSR_SEED_MAX];
} InsrLossFin;
/* Rows of loss_part the seeded backward of this call writes (one per block of its launch); 0 when
 * the backward the call routes to takes no in-kernel seeds (the fused tile-split path of value jets and
 * the saved-stream jet_fb sweep do; the two-kernel, split-bf16 resident and recompute paths, the fused
 * path of gradient / Laplacian jets and jet_fb blocks of more than 24 tiles do not). */
int insr_jet_bwd_seed_rows(long n_points, int d_in, int d_out, int num_hidden, int width, int mode);
/* The backward's first launch with seeds: the fused tile-split path (insr_siren_jet_bwd: partial rows
 * into `work`, summed by insr_reduce_partials_fin / insr_adam_step_partials_fin) or the jet_fb sweep
 * (insr_siren_jet_bwd_grad_adam phase 1 into `work`, phase 2 by insr_siren_jet_bwd_grad_adam_fin).
 * A stream with seeds has its adjoint pointer NULL; 1 <= n_seeds <= INSR_SEED_MAX. */
int insr_siren_jet_bwd_seeded(const float* x, long n_points, int d_in, int d_out, int num_hidden, int width, int mode,
                              const float* params, const float* act, const float* gy, const float* gdy,
                              const float* glap, const InsrSeed* seeds, int n_seeds, float* loss_part, float* work,
                              void* stream);
int insr_reduce_partials_fin(const float* partial, int n_blocks, long count, long stride, float* grad, int accumulate,
                             const InsrLossFin* fin, void* stream);
int insr_adam_step_partials_fin(const float* partial, int nb, long stride, float* grad, int accumulate, float* params,
                                float* exp_avg, float* exp_avg_sq, long count, const int* shape, float* opt_state,
                                float beta1, float beta2, float eps, const float* loss, int patience,
                                const InsrLossFin* fin, void* stream);
int insr_siren_jet_bwd_grad_adam_fin(const float* x, long n_points, int d_in, int d_out, int num_hidden, int width,
                                     int mode, float* params, float* work, float* grad, int accumulate, float* exp_avg,
                                     float* exp_avg_sq, float* opt_state, float beta1, float beta2, float eps,
                                     const float* loss, int patience, const InsrLossFin* fin, void* stream);

/*
 * Singular-value energies of the elasticity model (elasticity/model.py:143-163):
 *   out = sum_points [ ratio_arap sum_i (s_i - 1)^2 + ratio_volume (prod_i s_i - 1)^2 ],
 * s = singular values of each d x d block of J (n blocks, row-major, d = 2 or 3).
 * Forward: deterministic reduction (more than 1024 points: partials in `work`,
 * insr_svd_energy_work_floats() floats, combined by a second one-block launch).
 * Backward: gJ = gout[0] * U diag(dE/ds) V^T per block (torch.svd's gradient),
 * the SVD recomputed in registers (2x2 closed form, 3x3 one-sided Jacobi).
 */
long insr_svd_energy_work_floats(void);
int insr_svd_energy_fwd(const float* J, long n, int d, float ratio_arap, float ratio_volume, float* out,
                        float* work, void* stream);
int insr_svd_energy_bwd(const float* J, long n, int d, float ratio_arap, float ratio_volume, const float* gout,
                        float* gJ, void* stream);

/*
 * The elastodynamics energy of one elasticity iteration in ONE launch, with its gradient
 * for a unit seed (elasticity/model.py:131-186, elasticity/losses.py:6-20 and the 2-D case
 * of :22-39).  Replaces the jacobian + torch.svd + ~20 aten launches per direction of the
 * reference's energy, and insr_svd_energy_fwd/bwd + the torch terms here.
 * Rows [0, n) of f / J are the interior points x (q = f + x, q_prev = f_prev + x, q_pp =
 * f_pp + x, qdot = (q - q_prev) / dt); rows [row_l, row_l + n_l) and [row_r, row_r + n_r)
 * the fixed points of the positional constraints.  Terms (ratio[t] = 0 switches one off):
 *   ARAP            ratio * sum (s_i - 1)^2          s = singular values of J + I
 *   VOLUME          ratio * sum (prod s_i - 1)^2
 *   KINEMATICS      ratio * sum (qdot - qdot_prev)^2, qdot_prev = (q_prev - q_pp) / dt
 *   EXTERNAL        -dt * sum qdot . ext               (ratio: on / off)
 *   CONSTRAINT      ratio * sum |f(x_l)|^2
 *   CONSTRAINT_RIGHT ratio * sum |f(x_r) - target|^2  (target = +-offset)
 *   COLLISION       -dt * sum_{q_z < h} qdot_z ratio (h - q_z)   (plane, z = last coordinate)
 *   SPHERE          d = 2: -dt * sum_{|q - c| < R} qdot . ratio |q - c| dir
 *                   d = 3: -dt * ratio * (sum_{|q - c| < R} |q - c|) * (sum_{|q - c| < R} qdot . dir)
 *                   (elasticity/losses.py:22-39: in 3-D the reference's dist[:, None, None] * dir
 *                   broadcasts to (K, K, 3), a product of two sums; its gradient needs both sums,
 *                   so the launch adds a second pass over the interior rows when d = 3)
 * *out = the terms of order[0 .. n_order) added in that order (cfg.energy); terms[t] = term t
 * (terms may be NULL).  gf (rows, d) / gJ (rows, d, d) (either may be NULL): d out[0] / d f, d out[0] / dJ,
 * zeros on rows no term reads.  Each term's sum is reduced in a fixed order; work:
 * insr_elastic_work_floats() floats, zero-initialised once (the launch leaves its ticket zero).
 */
#define INSR_EL_ARAP 0
#define INSR_EL_VOLUME 1
#define INSR_EL_KINEMATICS 2
#define INSR_EL_EXTERNAL 3
#define INSR_EL_CONSTRAINT 4
#define INSR_EL_CONSTRAINT_RIGHT 5
#define INSR_EL_COLLISION 6
#define INSR_EL_SPHERE 7
#define INSR_EL_TERMS 8
typedef struct InsrElastic {
  int d;               /* 2 or 3 */
  int n_order;         /* terms in order[] */
  long n;              /* interior rows */
  long rows;           /* rows of f / J / gf / gJ */
  const float* f;      /* (rows, d) trainable field */
  const float* J;      /* (rows, d, d) its Jacobian (no identity); NULL without ARAP / VOLUME */
  const float* x;      /* (n, d) interior points */
  const float* f_prev; /* (n, d) */
  const float* f_pp;   /* (n, d) */
  float dt;
  float ratio[INSR_EL_TERMS];
  float ext[3];
  float target[3];
  float plane_height;
  float center[3];
  float radius;
  long row_l, n_l, row_r, n_r;
  int order[INSR_EL_TERMS];
  float* out;          /* 1 float: the total */
  float* terms;        /* INSR_EL_TERMS floats, or NULL */
  float* gf;
  float* gJ;
} InsrElastic;
long insr_elastic_work_floats(void);
int insr_elastic_energy(const InsrElastic* e, float* work, void* stream);

/*
 * Data-parallel collective (one process per GPU): the single sum all-reduce per optimiser
 * step of the flat gradients (+ loss scalars) -- what BaseModel._dp_sync does through
 * torch.distributed (backend "nccl" = RCCL), for hosts without PyTorch.  RCCL is loaded at
 * run time (the copy PyTorch already loaded, if any).
 *   rank 0: insr_comm_unique_id(id) -> share the insr_comm_id_bytes() bytes -> every rank:
 *   insr_comm_init(&comm, rank, world, id); per step insr_comm_allreduce_sum(comm, buf, n,
 *   stream) (in place, asynchronous on `stream`); insr_comm_destroy(comm) at the end.
 * Replaces: the gradient averaging a DDP port of base/baseModel.py:73-81 would add.
 */
int insr_comm_available(void);
long insr_comm_id_bytes(void);
int insr_comm_unique_id(void* id_out);
int insr_comm_init(void** comm, int rank, int world, const void* id);
int insr_comm_allreduce_sum(void* comm, float* buf, long count, void* stream);
int insr_comm_destroy(void* comm);

/*
 * Collocation draws of one phase iteration in ONE launch: n_boxes boxes of points in
 * dim (1..3) dimensions, box k = boxes[k].n points with coordinate j uniform in
 * [lo[j], hi[j]), written row-major (n, dim) to boxes[k].out. One Philox-4x32-10
 * stream keyed by `seed`; `state` (insr_sampler_state_bytes, zero-initialised device
 * memory, one per stream of draws) holds the stream position, which the launch
 * advances itself -- a captured graph draws fresh points on every replay.
 * Replaces: sample_random + sample_boundary2D_separate (base/sampling.py:14-64) as
 * called by the phases (fluid/model.py:74,90-91,105,116-117,129,135-136).
 */
#define INSR_MAX_BOXES 8
typedef struct InsrBox {
  float* out;   /* (n, dim) */
  long n;       /* points */
  float lo[3];  /* per coordinate */
  float hi[3];
} InsrBox;
long insr_sampler_state_bytes(void);
int insr_sample_boxes(const InsrBox* boxes, int n_boxes, int dim, unsigned long long seed, void* state,
                      void* stream);
/*
 * The draws of `reps` consecutive iterations in ONE launch (a hipGraph that replays U iterations
 * draws all of their points up front): repetition r of box k writes boxes[k].n fresh points at
 * boxes[k].out + r * rep_strides[k] floats.  reps = 1 (rep_strides may be NULL) is
 * insr_sample_boxes.  Same stream, same distributions (base/sampling.py draw_ahead).
 */
int insr_sample_boxes_rep(const InsrBox* boxes, int n_boxes, int dim, int reps, const long* rep_strides,
                          unsigned long long seed, void* state, void* stream);

/*
 * One advection iteration's forward, residual and reverse in ONE launch (round 6; csrc/advect_iter.hip):
 * the reference's Advection1DModel._advect (advection/model.py:68-91) on a 1 -> 1 SIREN of width 64 and
 * num_hidden (1..3) hidden layers -- the draw of n interior points in [box_lo[0], box_hi[0]) and
 * n_band_half points in each of the two Dirichlet bands (boxes 1, 2: the stream, values and device
 * state advance of insr_sample_boxes with those three boxes, dim 1), the value + x-derivative jets of
 * the frozen field (prev_params) and the trainable one (params), the residual
 *   r = (u - u0) / dt + vel (u_x + u0_x) / 2 on the interior, u on the bands,
 * and the parameter gradient of  sum r_int^2 / main_total + sum u_band^2 / bc_total  as one partial row
 * per block into `partials` ([rows][stride], stride >= the parameter count, a multiple of 4) with the
 * blocks' loss sums into loss_part ([rows][INSR_SEED_MAX] scratch); the last block to finish writes the
 * two losses to losses[0] (main = sum r_int^2 / main_total) and losses[1] (bc).  `points` (n + 2
 * n_band_half floats, may be NULL) receives the drawn points.  Returns the row count (=
 * insr_advect1d_rows(n + 2 n_band_half)) or a negative INSR_E*.  The rows are summed -- with the Adam (+
 * plateau, reading losses[0]) update -- by insr_adam_step_partials (or insr_reduce_partials_strided): an
 * iteration is two launches.  Replaces:
 * sample_random / sample_boundary (base/sampling.py:14-30), MLP.forward + gradient (base/diff_ops.py:44-58)
 * of both fields, the loss expressions and loss.backward() (base/baseModel.py:73-78).
 */
long insr_advect1d_rows(long n_points);
int insr_advect1d_iteration(const float* params, const float* prev_params, int num_hidden, int width, long n,
                            long n_band_half, const float* box_lo, const float* box_hi, float dt, float vel,
                            float main_total, float bc_total, unsigned long long seed, void* sampler_state,
                            float* points, float* partials, long stride, float* loss_part, float* losses,
                            void* stream);

#ifdef __cplusplus
}
#endif
#endif /* INSR_SIREN_H */
