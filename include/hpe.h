/* hpe.h — C ABI of libhpe.so, the MI355X (gfx950) head-pose regression hot path.
 *
 * The reference (Maaz77/Head-Pose-Estimation-Model) has no native code and no FFI: its boundary is
 * the Python/Keras API at the call sites below.  This ABI is what that Keras layer
 * bottoms out in once TF's CPU kernels are replaced; the Python host package
 * (head-pose-estimation-model_amd/hpe) binds it with ctypes and keeps the reference's surface.
 *
 *   hpe_program_create / _destroy   replaces keras.Model construction + compile
 *                                   (Model-96/train_96.py:65-110, Model-88/train_88.py:66-253,
 *                                    Model-88/attention_model.py:16-169): a compiled "row program"
 *                                    (per-position op list over a tile of rows kept in LDS)
 *   hpe_forward                     replaces model.predict (Model-96/test.py:34) and the forward of
 *                                   model.evaluate (train_96.py:186-187)
 *   hpe_train_step                  replaces one step of model.fit (train_96.py:175-183,
 *                                   train_88.py:355-363): forward + MSE + backward, per-workgroup
 *                                   gradient partials into the workspace
 *   hpe_reduce                      sums the per-workgroup partials into one flat gradient
 *                                   (the buffer RCCL all-reduces across ranks)
 *   hpe_optim_step                  replaces optimizer.apply_gradients of Keras' legacy SGD / Adam /
 *                                   Adamax (train_96.py:99-103, train_88.py:323) + the L2 penalty
 *                                   gradient of kernel_/bias_regularizer (train_96.py:78-79,90-91)
 *
 * Conventions: every buffer is a caller-owned DEVICE pointer (fp32 unless noted); every call is
 * stream-ordered on the hipStream_t passed as `stream` (0 = null stream) and never synchronises,
 * allocates or frees (graph-capturable).  Return value 0 = OK; otherwise hpe_last_error() (thread
 * local) holds the message.  Handles are not thread-safe; one per device.
 */
#ifndef HPE_H
#define HPE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hpe_program hpe_program;

/* Error codes */
#define HPE_OK 0
#define HPE_EINVAL 1   /* bad argument / shape (the Python layer raises ValueError) */
#define HPE_ERUNTIME 2 /* HIP runtime failure (RuntimeError) */

/* Optimizer kinds (Keras legacy optimizers) */
#define HPE_OPT_SGD 0
#define HPE_OPT_ADAM 1
#define HPE_OPT_ADAMAX 2

/* Create a program from the int32 word stream produced by hpe/compiler.py (layout documented in
 * csrc/hpe_prog.h).  Copies the words to device memory owned by the handle. */
int hpe_program_create(const int32_t *words, int64_t n_words, hpe_program **out);
int hpe_program_destroy(hpe_program *prog);

/* Number of workgroups a launch over n_rows rows uses, and the workspace bytes hpe_train_step
 * needs for it: grid x (n_params + 4) floats of per-workgroup partials. */
int hpe_launch_grid(const hpe_program *prog, int64_t n_rows);
size_t hpe_workspace_size(const hpe_program *prog, int64_t n_rows);

/* Forward over n_images images of P positions each (rows = n_images * P, channels-last rows of
 * C_in floats).  image_index (int32, may be NULL) gathers images: row r reads image
 * image_index[r / P].  y: n_images * P * C_out floats, channel order yaw, pitch, roll. */
int hpe_forward(const hpe_program *prog, const float *params, const float *params_t,
                const float *x, int64_t n_images, int32_t P, const int32_t *image_index,
                float *y, void *stream);

/* One training (or, with a program compiled for evaluation, loss-only) pass.  y_true: per-image
 * labels [n_images_total][C_out] indexed like x.  image_offset: global index of this rank's first
 * image (dropout hash).  inv_count: 1 / (global rows * C_out), the MSE normaliser.  workspace:
 * hpe_workspace_size() bytes; receives per-workgroup partial gradients and [sum e^2, sum |e|]. */
int hpe_train_step(const hpe_program *prog, const float *params, const float *params_t,
                   const float *x, const float *y_true, int64_t n_images, int32_t P,
                   const int32_t *image_index, int64_t image_offset, float inv_count,
                   uint64_t dropout_seed, void *workspace, void *stream);

/* hpe_train_step with the caller's bound on max |x| over the rows the launch reads (0 = unknown).
 * The fused kernels compute the GEMMs on an fp16 split whose data side holds |x| < 64 and hand a launch
 * whose split overflowed to an exact-fp32 twin launched behind it; with x_bound in (0, 64) the twin
 * cannot be needed and is not launched (fit bounds its resident dataset once per call). */
int hpe_train_step_bounded(const hpe_program *prog, const float *params, const float *params_t,
                           const float *x, const float *y_true, int64_t n_images, int32_t P,
                           const int32_t *image_index, int64_t image_offset, float inv_count,
                           uint64_t dropout_seed, float x_bound, void *workspace, void *stream);

/* grad[i] = sum over workgroups of workspace partials, i < n_params + 4 (fixed order). */
int hpe_reduce(const hpe_program *prog, int64_t n_rows, const void *workspace, float *grad,
               void *stream);

/* Keras legacy optimizer step on the flat parameter vector:
 *   g = grad[i] * grad_scale + 2 * l2[i] * w[i]
 *   SGD:    w -= lr g
 *   Adam:   m += (g - m)(1-b1); v += (g^2 - v)(1-b2); w -= alpha m / (sqrt(v) + eps),
 *           alpha = lr sqrt(1-b2^t) / (1-b1^t)
 *   Adamax: m += (g - m)(1-b1); v = max(b2 v, |g|); w -= lr/(1-b1^t) m / (v + eps)
 * t = iter (1-based).  tpos[i] >= 0 mirrors the new w[i] into params_t[tpos[i]] (the transposed
 * copy the backward GEMMs read).  grad holds n + 4 floats (the step's [sum e^2, sum |e|] follow
 * the gradient).  stats receives [grad[n], grad[n+1], reg_0 .. reg_{grid-1}] where reg_b is block
 * b's share of sum l2[i] w[i]^2 on the pre-update weights (the Keras regularisation loss). */
int hpe_optim_step(int32_t kind, float lr, float beta_1, float beta_2, float epsilon, int64_t iter,
                   float grad_scale, float *params, float *params_t, float *m, float *v,
                   const float *grad, const float *l2, const int32_t *tpos, int64_t n,
                   float *stats, void *stream);
/* Blocks hpe_optim_step launches (stats holds 2 + this many floats). */
int hpe_optim_grid(int64_t n);

/* hpe_reduce followed by hpe_optim_step in ONE launch, for a single rank (no all-reduce between
 * them): grad receives exactly what hpe_reduce writes (bit-identical: same summation order), the
 * parameters / moments / stats exactly what hpe_optim_step then writes.  n must equal the program's
 * trained-parameter count.  Used by the per-step fit path at small launch grids (P = 1 batches). */
int hpe_reduce_optim_step(const hpe_program *prog, int64_t n_rows, const void *workspace, float *grad,
                          int32_t kind, float lr, float beta_1, float beta_2, float epsilon, int64_t iter,
                          float grad_scale, float *params, float *params_t, float *m, float *v,
                          const float *l2, const int32_t *tpos, int64_t n, float *stats, void *stream);

/* One epoch of model.fit's per-step path for a single rank, the step loop in C (replaces the
 * Python step loop of Keras fit, train_96.py:175-183, for programs the whole-epoch kernel does not
 * take: P > 1 maps, batches above its limit, every graph the fused kernels do not cover).  For
 * s = 0 .. ceil(n / batch) - 1 with rows perm[s*batch .. min(n, (s+1)*batch)): hpe_train_step_bounded
 * (dropout seed seed_base + iter0 + 1 + s, inv_count = (float)(1.0 / (rows * P * 3)), x_bound), then
 * hpe_reduce_optim_step when hpe_launch_grid <= 16, else hpe_reduce + hpe_optim_step, with iteration
 * iter0 + 1 + s and stats + s * stats_stride — the launches fit issues from Python, bit-identical.
 * Each stats row receives hpe_optim_step's [sse, sae, reg_0 .. reg_{grid-1}]: stats_stride must be
 * >= 2 + hpe_optim_grid(n_train) (HPE_EINVAL otherwise), stats holds ceil(n / batch) rows. */
int hpe_fit_steps(const hpe_program *prog, float *params, float *params_t, float *m, float *v,
                  const float *l2, const int32_t *tpos, int64_t n_train, const float *x,
                  const float *y_true, const int32_t *perm, int64_t n, int32_t batch, int32_t P,
                  float x_bound, int32_t kind, float lr, float beta_1, float beta_2, float epsilon,
                  uint64_t seed_base, int64_t iter0, void *workspace, float *grad, float *stats,
                  int32_t stats_stride, void *stream);

/* One epoch of a DATA-PARALLEL rank's fit with the step loop in C (replaces the Python step loop of
 * hpe/model.py's distributed fit; the reference's loop: train_96.py:175-183).  Per step s over rows
 * perm[b0 .. b0 + nb) of the global batch (b0 = s * batch): this rank's share [r0, r1) with
 * r0 = b0 + nb * rank / world, r1 = b0 + nb * (rank + 1) / world; hpe_train_step_bounded on it
 * (img_off = r0 - b0, inv_count = (float)(1.0 / (nb * P * 3)): the GLOBAL count) + hpe_reduce into
 * grad (n_train + 4 floats; zeroed when the share is empty), then allreduce(grad, n_train + 4,
 * stream, user) — the caller's sum over ranks, e.g. an RCCL all-reduce on that stream; non-zero
 * aborts with HPE_ERUNTIME — then hpe_optim_step with iteration iter0 + 1 + s into
 * stats + s * stats_stride (stats_stride >= 2 + hpe_optim_grid(n_train)).  Bit-identical to the
 * per-step launches issued one by one.  steps_done (may be NULL) receives the number of steps whose
 * optimizer update was issued, also when the epoch stops early on an error (the caller advances its
 * iteration count by it). */
typedef int (*hpe_allreduce_fn)(float *buf, int64_t n, void *stream, void *user);
int hpe_fit_steps_dp(const hpe_program *prog, float *params, float *params_t, float *m, float *v,
                     const float *l2, const int32_t *tpos, int64_t n_train, const float *x,
                     const float *y_true, const int32_t *perm, int64_t n, int32_t batch, int32_t P,
                     float x_bound, int32_t kind, float lr, float beta_1, float beta_2, float epsilon,
                     uint64_t seed_base, int64_t iter0, void *workspace, float *grad, float *stats,
                     int32_t stats_stride, int32_t rank, int32_t world, hpe_allreduce_fn allreduce,
                     void *user, int64_t *steps_done, void *stream);

/* Native RCCL all-reduce for hpe_fit_steps_dp on GPU ranks (csrc/hpe_rccl.hip; librccl opened at
 * run time): replaces the caller's per-step hook (e.g. a torch.distributed callback, one
 * interpreter re-entry per step) by an RCCL sum enqueued on the step's own stream.  Rank 0 calls
 * hpe_rccl_unique_id, the caller broadcasts the HPE_RCCL_ID_BYTES bytes to every rank, each rank
 * calls hpe_rccl_comm_init on its current device; then hpe_fit_steps_dp(..., allreduce =
 * hpe_rccl_allreduce, user = the communicator, ...).  hpe_rccl_available: 1 when librccl loads. */
#define HPE_RCCL_ID_BYTES 128
int hpe_rccl_available(void);
int hpe_rccl_unique_id(void *id_out);
int hpe_rccl_comm_init(const void *id, int32_t nranks, int32_t rank, void **comm_out);
int hpe_rccl_comm_destroy(void *comm);
int hpe_rccl_allreduce(float *buf, int64_t n, void *stream, void *comm);

/* ---------------------------------------------------------------------------------------------
 * One whole epoch of model.fit in ONE launch (csrc/hpe_fit.hip) — replaces the per-step loop of
 * Keras fit (train_96.py:175-183, train_88.py:355-363) for the reference's own regime: 1x1 maps
 * (P = 1), the 2-layer create_model family (programs of kind mlp2 compiled for training), one rank.
 * Equivalent to, for s = 0 .. ceil(n / batch) - 1 with rows perm[s*batch .. min(n, (s+1)*batch)):
 *   hpe_train_step (dropout_seed = seed_base + iter0 + 1 + s, inv_count = 1 / (rows * 3)),
 *   hpe_reduce, hpe_optim_step(kind, lr, beta_1, beta_2, epsilon, iter0 + 1 + s, 1.0)
 * with alpha[s] the optimizer step size hpe_optim_step derives for that iteration (lr for SGD,
 * lr sqrt(1-b2^t)/(1-b1^t) for Adam, lr/(1-b1^t) for Adamax; device array of ceil(n / batch)).
 * params / params_t / m / v are updated in place; stats[s * stats_stride + ...] receives the
 * step's [sum e^2, sum |e|, reg_0 .. reg_{G-1}] (G = ceil(F / 32) workgroups; the regularisation
 * loss on the pre-update weights is the sum of the reg_g).  exact != 0 runs exact-fp32 MFMA GEMMs.
 * workspace: hpe_fit_workspace_size bytes; after the launch its int word [1] holds flags
 * (1: a split accumulator was non-finite — rerun the epoch with exact = 1 from the saved state;
 * 2: the per-step workgroup exchange timed out — the workgroups may have stopped at different
 * steps, so restore params / m / v and run the epoch per step).  hpe_fit_supported: 1 if program
 * + batch qualify: F <= 1024 (G <= 32), batch <= 512, the exchange table G * batch * 3 floats
 * within 9,216 (batch <= 256) or 25,600 (batch 257..512), and all G workgroups co-resident (one
 * per CU, G <= CUs / 8); 0 otherwise (and without a device).  Env HPE_FIT_FORCE_TIMEOUT=1 (tests)
 * raises flag 2 at the first exchange. */
int hpe_fit_supported(const hpe_program *prog, int32_t batch);
size_t hpe_fit_workspace_size(const hpe_program *prog, int32_t batch);
int hpe_fit_epoch(const hpe_program *prog, float *params, float *params_t, float *m, float *v,
                  const float *l2, const int32_t *tpos, const float *x, const float *y_true,
                  const int32_t *perm, int64_t n, int32_t batch, int32_t kind, float lr, float beta_1,
                  float beta_2, float epsilon, const float *alpha, uint64_t seed_base, int64_t iter0,
                  float *stats, int32_t stats_stride, int32_t exact, void *workspace, void *stream);

/* ---------------------------------------------------------------------------------------------
 * BlazeFace backbone — replaces the TF call on the fused BlazeFace+regressor
 * graph, `self.model.predict(...)` at BlazePoser/blazeFaceDetectorH5.py:272, for a whole batch.
 * words: the plan hpe/blazeface.py builds from the unified model's model_config (csrc/hpe_prog.h
 * BFH_* / BFO_*); params: the plan's flat fp32 parameter vector (device).
 * images: (n_images, 128, 128, 3) NHWC fp32 in [-1, 1] (the detector's preprocessed input).
 * outs: six device pointers (host array), in the unified model's output order:
 *   [0] classificators_1 (n,512,1)  [1] classificators_2 (n,384,1)
 *   [2] regressors_1 (n,512,16)     [3] regressors_2 (n,384,16)
 *   [4] re_lu_10 tap (n,16,16,88)   [5] re_lu_15 tap (n,8,8,96)
 * The two pose regressors of the unified model (`model` on re_lu_10, `model_10` on re_lu_15) run
 * on the taps through hpe_forward (programs compiled with P = 256 and P = 64).
 * workspace: hpe_blazeface_workspace_size(h, n_images) bytes of device memory. */
typedef struct hpe_blazeface hpe_blazeface;
int hpe_blazeface_create(const int32_t *words, int64_t n_words, hpe_blazeface **out);
int hpe_blazeface_destroy(hpe_blazeface *h);
size_t hpe_blazeface_workspace_size(const hpe_blazeface *h, int64_t n_images);
int hpe_blazeface_forward(const hpe_blazeface *h, const float *params, const float *images,
                          int64_t n_images, float *const *outs, void *workspace, void *stream);

/* Detector post-processing of the unified graph for a batch of frames,
 * replacing blazeFaceDetector.filterDetections / extractDetections / filterWithNonMaxSupression
 * (BlazePoser/blazeFaceDetectorH5.py:284-357) per frame:
 *   keep logit > score_logit_threshold (fp32; the reference's log(t/(1-t))), score = sigmoid (fp32),
 *   decode boxes / 6 keypoints against the 896 SSD anchors in fp64, greedy NMS with
 *   tf.image.non_max_suppression semantics (IoU in fp32, suppress iff IoU > iou_threshold, at most
 *   max_faces kept), and gather each kept detection's pose from its 16x16 / 8x8 regressor cell.
 * Inputs (device): cls0 (n,512), cls1 (n,384), loc0 (n,512,16), loc1 (n,384,16), pose0 (n,16,16,3),
 * pose1 (n,8,8,3).  Outputs (device, per frame max_faces slots, the first count[i] valid, in NMS
 * selection order): det_index int32, scores f32, boxes f64 [x1,y1,x2,y2], keypoints f64 [6][2],
 * poses f32 [yaw, pitch, roll]. */
int hpe_detect(const float *cls0, const float *cls1, const float *loc0, const float *loc1,
               const float *pose0, const float *pose1, int64_t n_images, float score_logit_threshold,
               float iou_threshold, int32_t max_faces, int32_t *count, int32_t *det_index, float *scores,
               double *boxes, double *keypoints, float *poses, void *stream);

/* Feature-dataset extraction (the *_features_88|96_<t>_<k>.npz files of
 * FeatureMaps-Datasets/, whose extractor is outside the reference, JoinModels.py:114 taps re_lu_10 /
 * re_lu_15): for the first k kept detections of each frame (hpe_detect outputs), the regressor input
 * that detection's pose was computed from, following the pose gather at blazeFaceDetectorH5.py:342-353
 * — d < 512: tap0 (n,16,16,c0) cell d/2; else tap1 (n,8,8,c1) cell (d-512)/6.  Outputs (device):
 * feat0 (n,k,c0), feat1 (n,k,c1) (the other tap's row zero), src (n,k) int32 0 / 1 / -1 (empty). */
int hpe_gather_features(const int32_t *count, const int32_t *det_index, int64_t n_images, int32_t max_faces,
                        int32_t k, const float *tap0, int32_t c0, const float *tap1, int32_t c1, float *feat0,
                        float *feat1, int32_t *src, void *stream);

const char *hpe_last_error(void);

/* Build stamp: "src=<sha256/16 of the library's sources> git=<commit>[-dirty]" (csrc/Makefile).  The
 * Python binding recomputes the source hash from the tree it runs in and refuses a library built
 * from other sources, so a run's kernels are provably the checkout's. */
const char *hpe_build_id(void);

/* Dominant-kernel timing (bench.py's roofline): hpe_kernel_timing(capacity) turns timing on for
 * the next `capacity` program launches (0 turns it off): hpe_forward / hpe_train_step record a HIP
 * event pair on their stream around the launch's dominant kernel only (the fp16-split kernel, not
 * its early-exit exact twin, nor hpe_reduce).  hpe_kernel_times waits for the recorded pairs and
 * writes their elapsed milliseconds to ms[0 .. n); returns n (<= max): the leading run of pairs
 * whose launch has finished recording (a launch another host thread has not returned from yet
 * ends the run). */
int hpe_kernel_timing(int32_t capacity);
int hpe_kernel_times(float *ms, int32_t max);

/* Diagnostics (race screens; synchronises the device, so not for the hot path): out[0] = the
 * program's last launch epoch, out[1 .. 16] its guard ring (word e % 16 holds e when launch e's
 * fp16-split kernel flagged a non-finite value and its exact-fp32 twin recomputed the step),
 * out[17 .. 32] reserved per ring slot for which check fired (no current kernel writes them: 0). */
int hpe_guard_peek(const hpe_program *prog, int32_t *out);

/* Precision of the regressor GEMMs (process-wide; returns the previous setting).  Default 0: the
 * fused kernels run their fp32 GEMMs as three fp16 MFMAs per product (hi/lo split, fp32
 * accumulate, ~2^-22 relative per product; csrc/hpe_common.h mfma3), and a launch whose split
 * overflows fp16 (|value| >= 65504) is recomputed by the exact-fp32 kernel automatically.
 * 1: exact-fp32 MFMA (v_mfma_f32_32x32x2_f32) only.  The environment variable HPE_EXACT_FP32=1
 * sets the initial value. */
int hpe_set_exact_fp32(int on);

/* Diagnostics: out[i] = the fused regressor kernels' layer-1 activation `act` (ACT_* of
 * csrc/hpe_prog.h) of z[i], as they evaluate it (csrc/hpe_dev.h act1_f).  fast = 1: the fp16-split
 * kernels' form (tanh: fast_tanh5, absolute error <= 2^-22); fast = 0: the exact-fp32 kernels'
 * (tanh: tanhf).  Device pointers, n floats; asynchronous on `stream`. */
int hpe_act_probe(int32_t act, int32_t fast, const float *z, float *out, int64_t n, void *stream);

/* Attention heads on H x W > 1 feature maps: the two stages that are not
 * row-local.  Replace the TF kernels behind GlobalAveragePooling2D -> Dense -> Dense -> Multiply
 * (Model-88/attention_model.py:34-38, :78-82) and behind MultiHeadAttention's softmax(QK^T)V over
 * the H*W tokens of each image (attention_model.py:52-55).
 *
 * hpe_se_gate: x, xg [n_images * P][C] rows; w1 [C][U] (+ b1 [U], may be NULL), w2 [U][C]
 * (+ b2 [C]); act1 / act2 activation codes of csrc/hpe_prog.h (ACT_*).  xg = x * s[image].
 * hpe_mha: per row, in = [pass-through C | q H*D (pre-scaled by 1/sqrt(D)) | k H*D | v H*D]
 * (stride ld_in floats); out = [pass-through C | o H*D] (stride ld_out).  1 <= D <= 64. */
int hpe_se_gate(const float *x, float *xg, int64_t n_images, int32_t P, int32_t C, const float *w1,
                const float *b1, int32_t U, int32_t act1, const float *w2, const float *b2,
                int32_t act2, void *stream);
/* y[i][c] = mean over the P rows of image i of x (a terminal GlobalAveragePooling2D), C <= 256. */
int hpe_seg_mean(const float *x, float *y, int64_t n_images, int32_t P, int32_t C, void *stream);
int hpe_mha(const float *in, int32_t ld_in, int32_t C, float *out, int32_t ld_out,
            int64_t n_images, int32_t P, int32_t H, int32_t D, void *stream);
/* hpe_mha_xg: the same attention with the pass-through columns read from their own rows: qkv =
 * [q H*D (pre-scaled) | k H*D | v H*D] (stride ld_qkv), xg [n_images * P][C] contiguous; out =
 * [xg | o H*D] (stride ld_out).  The projection that feeds it then computes only q | k | v (no
 * identity block for xg: 2 * C * C fewer FLOPs and C fewer stored floats per row). */
int hpe_mha_xg(const float *qkv, int32_t ld_qkv, const float *xg, int32_t C, float *out, int32_t ld_out,
               int64_t n_images, int32_t P, int32_t H, int32_t D, void *stream);

/* hpe_attn_tail: the row-local tail of se_transformer_regr_head after the attention core
 * (Model-88/attention_model.py:56-72: residual Add of the attention output, LayerNorm, feed-forward
 * Dense -> Dense, residual Add, LayerNorm, 1x1 conv hidden -> 1x1 conv 3) in one kernel: reads xg
 * [n_rows][ld_xg >= C] and the attention output o [n_rows][ld_o >= H*D] (hpe_mha_xg with C = 0),
 * writes y [n_rows][3].  desc: 20 host int32 words (C, H*D, ff_dim, hidden, activations, the two
 * LayerNorm epsilons as float bits, the parameter buffer's size and vector offsets); w: the device
 * parameter buffer hpe/spatial.py:_attn_tail prepares (weights in MFMA operand order, padded
 * vectors).  hpe_attn_tail_supported(desc): 1 when a kernel is compiled for these widths. */
int hpe_attn_tail_supported(const int32_t *desc);
int hpe_attn_tail(const float *xg, int32_t ld_xg, const float *o, int32_t ld_o, int64_t n_rows,
                  const int32_t *desc, const float *w, float *y, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* HPE_H */
