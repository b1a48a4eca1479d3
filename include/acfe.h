/*
 * acfe.h -- C ABI of the MI355X-native audio-classification front end + engine
 * ("acfe") that replaces the hot path of TheCacophonyProject/audio-training.
 *
 * Conventions (every entry point):
 *   - extern "C", plain pointers and sizes, no C++ / torch types.
 *   - Return 0 on success; < 0 on error: ACFE_E_INVAL for bad arguments,
 *     -(int)hipError_t for a HIP failure.  Nothing throws across the ABI.
 *   - Every buffer argument is caller-owned DEVICE memory unless the name ends
 *     in `_host`.  The library allocates only inside acfe_plan_create (twiddles,
 *     window, banded mel filterbank), freed by acfe_plan_destroy.
 *   - Every compute call takes the hipStream_t it is ordered on (passed as
 *     void*; NULL = the default stream), is asynchronous and reentrant, and
 *     never synchronises the device (graph-capturable).
 *   - Tensor layouts: raw audio [B][N] fp32 with a clip stride (elements
 *     between consecutive clips); features [B][T][M] ("BTM") or [B][M][T]
 *     ("BMT" == NHWC with H=M, W=T, C=1, the model input of
 *     resnet/wr_resnet*.py); activations NHWC; conv weights KRSC.
 *
 * Reference interfaces replaced (file:line in the reference repository):
 *   acfe_mel_filterbank    custommel.py:18-54        mel_f(sr,n_mels,fmin,fmax,n_fft,break_freq)
 *   acfe_plan_create       tfdataset.py:430-460      MEL_WEIGHTS / NFFT / HOP_LENGTH globals
 *   acfe_normalize_stats   tfdataset.py:1916-1934    normalize (reductions)
 *   acfe_normalize_apply   tfdataset.py:1916-1934    normalize (pointwise)
 *   acfe_mixup             tfdataset.py:930-955      mix_up (x blend; lambda drawn by caller)
 *   acfe_mel_fwd           tfdataset.py:2007-2059    raw_to_mel  (pad_end, power 2)
 *                          predict_utils.py:163-239  get_spect   (center, power 2)
 *                          tfdataset.py:1082-1090    spectrogram path (power 1)
 *   acfe_pcen_fwd          tfpcen.py:33-39,89-99     ExponentialMovingAverage + PCEN.call
 *   acfe_pcen_normalize    tfpcen.py:105-110         normalize_minmax (batch-global)
 *   acfe_pcen_bwd          gradient of the three above w.r.t. gain/bias/root/smooth
 */
#ifndef ACFE_H
#define ACFE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACFE_OK 0
#define ACFE_E_INVAL (-1000)
#define ACFE_E_NOMEM (-1001)

/* Framing of acfe_mel_fwd. */
#define ACFE_PAD_END 0            /* tf.signal.stft(pad_end=True): frames = ceil(N/hop)          */
#define ACFE_PAD_CENTER_CONSTANT 1 /* librosa.stft(center=True, pad_mode="constant") (>=0.10)   */
#define ACFE_PAD_CENTER_REFLECT 2  /* librosa.stft(center=True, pad_mode="reflect")  (<0.10)     */

#define ACFE_LAYOUT_BTM 0
#define ACFE_LAYOUT_BMT 1

#define ACFE_DTYPE_F32 0
#define ACFE_DTYPE_BF16 1

typedef struct acfe_plan_s* acfe_plan_t;

/* Library version (major*10000 + minor*100 + patch). */
int acfe_version(void);

/* Last HIP error string (thread-local), for diagnostics. */
const char* acfe_last_error(void);

/* Host CRC-32C (Castagnoli) of n bytes continuing from `crc` (0 to start):
 * the checksum of the TFRecord framing written by tf.io.TFRecordWriter
 * (audiowriter.py:259-277) and read by tf.data.TFRecordDataset
 * (tfdataset.py:212-214).  No GPU involved. */
uint32_t acfe_crc32c(const void* data, size_t n, uint32_t crc);

/* ---- Native TFRecord reader (host code; replaces tf.data.TFRecordDataset(
 * filenames, compression_type="GZIP") + ignore_errors(), tfdataset.py:212-226,
 * and the parse of read_tfrecord, tfdataset.py:1005-1060).  Reentrant; one
 * reader per thread.  Python calls these through ctypes, which releases the
 * GIL for the call, so reader threads inflate and parse in parallel. */
#define ACFE_E_IO (-1002)       /* file cannot be opened / read            */
#define ACFE_E_CORRUPT (-1003)  /* framing, CRC or protobuf error          */
typedef struct acfe_tfr_s* acfe_tfr_t;
/* Open a shard (compression 1 = GZIP, 0 = none): the file is read and
 * inflated whole into host memory owned by the reader. */
int acfe_tfr_open(const char* path, int compression, acfe_tfr_t* reader);
/* Next record: 1 and (*data_host, *len) pointing into the reader's buffer
 * (valid until close); 0 at a clean end; ACFE_E_CORRUPT on a truncated or
 * CRC-failing record (nothing after it is readable, as tf.data's
 * ignore_errors() ends the file there). */
int acfe_tfr_next(acfe_tfr_t reader, int check_crc, const uint8_t** data_host, uint64_t* len);
int acfe_tfr_close(acfe_tfr_t reader);
/* Fields of one tf.train.Example: the float_list of `float_key`
 * ("audio/raw" [144000] or "audio/spectogram" [2049*513]) -> *count floats,
 * copied to out_host when out_host != NULL and *count == n_out; the first
 * value of "audio/class/text" -> text_host (NUL-terminated, truncated to
 * text_cap).  Returns flags: 1 = float key present, 2 = copied and all
 * finite (the NaN/Inf filter of tfdataset.py:297), 4 = text present; or
 * ACFE_E_CORRUPT for a malformed message. */
int acfe_example_audio(const uint8_t* rec, uint64_t len, const char* float_key, float* out_host,
                       int64_t n_out, char* text_host, int text_cap, int64_t* count);

/* custommel.mel_f restated in C (float64 arithmetic, float32 result) into a
 * caller-owned HOST array out_host[n_mels][1 + n_fft/2]. */
int acfe_mel_filterbank(int sr, int n_mels, double fmin, double fmax, int n_fft,
                        double break_freq, float* out_host);

/* Create a front-end plan.  `mel_weights_host` is the dense [n_mels][1+n_fft/2]
 * float32 filterbank (as custommel.mel_f returns it) or NULL to compute it
 * with acfe_mel_filterbank(sr, n_mels, fmin, fmax, n_fft, break_freq).
 * n_fft must be a power of two in [256, 4096].  Allocates device memory on
 * the current device. */
int acfe_plan_create(int sr, int n_fft, int hop, int n_mels, double fmin, double fmax,
                     double break_freq, const float* mel_weights_host, acfe_plan_t* plan);
int acfe_plan_destroy(acfe_plan_t plan);
/* Number of frames the plan produces for an N-sample clip with pad_mode. */
int acfe_plan_num_frames(acfe_plan_t plan, int n_samples, int pad_mode);

/* Per-clip normalisation statistics: stats[b] = {min_b, max_b(x - min_b)}.
 * Clip b is x[b*clip_stride .. b*clip_stride + n). */
int acfe_normalize_stats(const float* x, int64_t clip_stride, int batch, int n,
                         float* stats, void* stream);
/* y[b][i] = ((x - min)/range + 1e-6 - 0.5) * 2, in that float32 order.
 * In place (y == x) is allowed when clip_stride == n. */
int acfe_normalize_apply(const float* x, int64_t clip_stride, int batch, int n,
                         const float* stats, float* y, void* stream);
/* mix_up on normalised inputs: y = norm(x1)*lam + norm(x2)*(1-lam), per row.
 * stats1/stats2 may be NULL (inputs already normalised). */
int acfe_mixup(const float* x1, const float* stats1, const float* x2, const float* stats2,
               const float* lam, int batch, int n, float* y, void* stream);
/* Row copies of the loader's device-resident clip pool (the shuffle buffer,
 * tfdataset.py:835-838): dst[dst_idx[i]][0..n) = src[src_idx[i]][0..n) for
 * i < count; a NULL index list is the identity.  Index lists are device int32
 * holding rows < src_rows / dst_rows (the caller checks them on the host
 * before the launch). */
int acfe_copy_rows(const float* src, int64_t src_stride, int64_t src_rows, const int* src_idx, float* dst,
                   int64_t dst_stride, int64_t dst_rows, const int* dst_idx, int count, int n, void* stream);

/* Fused framing -> periodic Hann -> n_fft real FFT (LDS radix-8/4 Stockham)
 * -> |X|^power (power 1 or 2) -> banded mel, for every frame of every clip.
 * If `stats` is non-NULL each clip is normalised on load (tfdataset.normalize).
 * out: layout ACFE_LAYOUT_BTM -> [B][T][M], ACFE_LAYOUT_BMT -> [B][M][T], fp32. */
int acfe_mel_fwd(acfe_plan_t plan, const float* raw, int64_t clip_stride, int batch, int n,
                 const float* stats, int pad_mode, int power, float* out, int layout,
                 void* stream);
/* n_fft = 4096 kernel of acfe_mel_fwd: 0 = two waves per frame (k_mel_w4),
 * f in 1..64 = one wave per frame walking f frames (k_mel_w5, bit-identical
 * output).  Initial value from the environment (ACFE_MEL_W5, default see
 * DESIGN.md); returns the previous setting, ACFE_E_INVAL out of range. */
int acfe_mel_w5_frames(int frames_per_wave);

/* Stored-spectrogram path (load_raw=False): mel = W . S^power of the magnitude
 * spectrogram each record holds, S = |librosa.stft| [n_bins][T] fp32 (clip b at
 * spec + b*clip_stride, frame-contiguous rows), through the plan's banded
 * filterbank; out [B][T][M] (layout 0) or [B][M][T] (layout 1).  Replaces the
 * per-example tf.tensordot(MEL_WEIGHTS, spectogram) of tfdataset.py:1082-1090
 * (power 1 there: the magnitude is kept for PCEN, :1085-1089). */
int acfe_mel_from_spec(acfe_plan_t plan, const float* spec, int64_t clip_stride, int batch, int n_bins, int T,
                       int power, float* out, int layout, void* stream);

/* PCEN forward on mel [B][T][M] fp32 (tfpcen.py:89-95):
 *   a_t = w x_t + (1-w) a_{t-1}, a_{-1} = x_0,  w = clip(smooth, 0, 1)
 *   y   = (x/(eps + a)^min(gain,1) + bias)^(1/max(root,1)) - bias^(1/max(root,1))
 * params: DEVICE float[4] = {gain, bias, root, smooth}; eps is a constant.
 * y is written UN-normalised as [B][M][T] fp32 (model layout).
 * minmax_partial: device float[2 * acfe_pcen_partials(batch, n_mels)]. */
int acfe_pcen_partials(int batch, int n_mels);
int acfe_pcen_fwd(const float* mel_btm, int batch, int t, int m, const float* params, float eps,
                  float* y_bmt, float* minmax_partial, void* stream);
/* normalize_minmax over the whole batch (tfpcen.py:105-110):
 *   out = 2*((y - mn)/(mx - mn)) - 1 written as fp32 or bf16 (out_dtype).
 * stats_out: device float[4] = {mn, mx, count(y==mn), count(y==mx)} (saved for
 * the backward).  When `scope_minmax` is non-NULL it overrides the reduction
 * with a caller-supplied {mn, mx} (e.g. all-reduced across replicas). */
int acfe_pcen_normalize(const float* y_bmt, int64_t count, const float* minmax_partial,
                        int n_partial, const float* scope_minmax, void* out, int out_dtype,
                        float* stats_out, void* stream);
/* Gradient of PCEN+normalize_minmax w.r.t. params {gain,bias,root,smooth}.
 * dout: [B][M][T] gradient w.r.t. the normalised output (fp32 or bf16).
 * workspace: device float[32 * acfe_pcen_partials(batch, n_mels)] (8-byte aligned).
 * dparams: device float[4] (overwritten). */
int acfe_pcen_bwd(const float* mel_btm, int batch, int t, int m, const float* params, float eps,
                  const float* stats, const void* dout, int dout_dtype, float* workspace,
                  float* dparams, void* stream);

/* ===================================================================== model
 * Replaces the Keras layers of resnet/wr_resnet.py:5-90 and
 * resnet/wr_resnet_bird.py:7-179 (Conv2D, BatchNormalization, ReLU, Add,
 * Dropout, MaxPool2D, AveragePooling2D, logmeanexp, GlobalAveragePooling2D,
 * Dense) and the loss / optimizer of audiomodel.py:1206-1240.
 * Activations NHWC (dtype ACFE_DTYPE_*), weights fp32 KRSC master copies. */

/* Packed-weight shape [rows_p][cols_p] for acfe_conv2d_pack_weights:
 * flip=0 -> forward operand [K pad][R*S*C pad]; flip=1 -> dgrad operand
 * [C pad][R*S*K pad] with the kernel rotated by 180 degrees. */
int acfe_conv2d_packed_shape(int K, int R, int S, int C, int dtype, int flip, int* rows_p, int* cols_p);
int acfe_conv2d_pack_weights(const float* w_krsc, int K, int R, int S, int C, int dtype, int flip,
                             void* out, void* stream);
/* All of a step's packings in one launch: descs = device array of n (<= 256)
 * records {const float* w; void* out; int64 begin; int K, R, S, C, flip,
 * rows_p, cols_p, pad} (56 B, the arguments of acfe_conv2d_pack_weights with
 * the record's first element in the concatenated index space [0, total),
 * begin ascending); dtype as acfe_conv2d_pack_weights, one for all records. */
int acfe_conv2d_pack_weights_batch(const void* descs, int n, long long total, int dtype, void* stream);
/* Rows of the per-channel statistics slab written by acfe_conv2d_fwd
 * (stats_partial: double[rows][2][rows_p of the forward packing]). */
int acfe_conv2d_stats_rows(long long M, int K);
/* Keras Conv2D forward (tf.keras.layers.Conv2D, NHWC): y[n,p,q,k] =
 * sum_{r,s,c} x[n, p*stride - pad_top + r, q*stride - pad_left + s, c] w[k,r,s,c] + bias[k].
 * Out-of-range taps read zero, so "same" needs only the top/left pads
 * (TF: pad_total = max((P-1)*stride + R - H, 0), pad_top = pad_total/2).
 * Optionally writes per-block {sum y, sum y^2} of the ROUNDED outputs for the
 * next BatchNormalization (stats_partial, may be NULL). */
int acfe_conv2d_fwd(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int R, int S,
                    int stride, int pad_top, int pad_left, int P, int Q, const float* bias, void* y,
                    int dtype, double* stats_partial, void* stream);
/* As acfe_conv2d_fwd, then Dropout(rate) of the output fused in the epilogue
 * (mask of acfe_dropout(seed) over the flat NHWC index; wr_resnet_bird.py:141
 * Dropout after branch 21); stats_partial then holds the dropped-out values. */
int acfe_conv2d_fwd_dropout(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int R, int S,
                            int stride, int pad_top, int pad_left, int P, int Q, const float* bias, void* y,
                            int dtype, double* stats_partial, float drop_rate, unsigned long long seed,
                            void* stream);
/* dX of the convolution above (wflip = flip=1 packing).  stride > 1 runs the
 * st x st sub-pixel phases as stride-1 convs of dY with the phase sub-kernels
 * (no zero insertion) and needs `workspace` of acfe_conv2d_dgrad_workspace
 * bytes (C * sizeof(dtype) a multiple of 16, dx 16-B aligned). */
long long acfe_conv2d_dgrad_workspace(int N, int P, int Q, int K, int C, int R, int S, int stride, int pad_top,
                                      int pad_left, int H, int W, int dtype);
int acfe_conv2d_dgrad(const void* dy, int N, int P, int Q, int K, const void* wflip, int C, int R, int S,
                      int stride, int pad_top, int pad_left, int H, int W, void* dx, int dtype,
                      void* workspace, void* stream);
/* acfe_conv2d_dgrad (stride 1, 3x3) whose dX is the output gradient of a
 * BatchNormalization (+ReLU) -- wr_resnet.py:56-80's bn2a / bn2b feeding
 * conv2a / conv2b -- with that BN's acfe_bn_bwd_reduce slab formed in the same
 * pass: x_bn = the BN input [N][H][W][C], scale / shift / mean / invstd its
 * acfe_bn_finalize outputs, part = [part_rows][2][C] for
 * acfe_bn_bwd_finalize_ex (nrows = part_rows).  _rows returns the slab rows,
 * or 0 when the fused form does not cover the shape (then: acfe_conv2d_dgrad +
 * acfe_bn_bwd_reduce).  Covered: C = 64 (any K % 64 == 0) and, since r06,
 * C = K = 128 (wr_resnet's stage-2 dgrads; environment ACFE_DGRADBN128=0
 * reports it uncovered, for A/B runs). */
int acfe_conv2d_dgrad_bn_rows(int N, int H, int W, int C, int K, int R, int S, int stride, int dtype);
int acfe_conv2d_dgrad_bn(const void* dy, int N, int P, int Q, int K, const void* wflip, int C, int R, int S,
                         int stride, int pad_top, int pad_left, int H, int W, void* dx, int dtype,
                         const void* x_bn, const float* scale, const float* shift, const float* mean,
                         const float* invstd, int relu, double* part, int part_rows, void* stream);
/* Kernel-variant switch for A/B checks and the parity tests: 1 (default, or
 * the ACFE_R64 environment variable) runs the K = 64 row-halo convolutions
 * (acfe_conv2d_fwd / _dropout / _bn / _add / _add_bn, acfe_conv2d_dgrad at
 * stride 1, acfe_conv2d_dgrad_bn) on the kernel that overlaps each tile's
 * epilogue with the next tile's MFMAs; 0 on the previous kernel (identical
 * results).  Returns the previous setting.  Not stream-ordered: set it
 * between launches. */
int acfe_conv_r64_enable(int on);
/* float count of the wgrad split-K workspace. */
long long acfe_conv2d_wgrad_workspace(int N, int H, int W, int C, int K, int R, int S, int P, int Q);
/* dW (fp32 KRSC) = beta*dW + sum_pixels dY (x) im2col(X). */
int acfe_conv2d_wgrad(const void* x, int N, int H, int W, int C, const void* dy, int K, int R, int S,
                      int stride, int pad_top, int pad_left, int P, int Q, float* dw, float beta, int dtype,
                      float* workspace, void* stream);
/* The wgrad of a bf16 3x3 stride-1 "same" conv whose output feeds [Dropout ->]
 * BatchNormalization (+ReLU) -- resnet/wr_resnet.py:58-71 (conv2a -> Dropout ->
 * bn2b -> ReLU), resnet/wr_resnet_bird.py:139-154 (conv21 -> Dropout -> bn2b)
 * -- taking that BN's OUTPUT gradient gy and its input u_bn: the conv output
 * gradient dy = acfe_bn_bwd_apply_ex(gy, u_bn, scale, shift, relu, coef, add,
 * drop_rate, seed, ...) is formed while the wgrad stages it (no separate apply
 * pass; add != NULL: the residual form -- the conv's output z = (ReLU)(conv +
 * shortcut) is the next block's bn2a input (resnet/wr_resnet.py:82-89), add
 * its identity shortcut's gradient, relu bit 1 the ReLU of z; no dropout)
 * pass over the tensor), written to dy (bit-identical to the apply pass's;
 * the dgrad reads it next) and summed per channel into sums
 * [acfe_conv2d_wgrad_bnbwd_rows][2][K] (finalize with
 * acfe_channel_sum_finalize: the conv bias gradient).  dw / beta / workspace as
 * acfe_conv2d_wgrad.  _rows: 0 when the shape is not covered (then
 * acfe_bn_bwd_apply_ex + acfe_conv2d_wgrad). */
int acfe_conv2d_wgrad_bnbwd_rows(int N, int H, int W, int C, int K);
int acfe_conv2d_wgrad_bnbwd(const void* x, int N, int H, int W, int C, const void* gy, const void* u_bn, int K,
                            const float* scale, const float* shift, int relu, const float* coef, const void* add,
                            float drop_rate, unsigned long long seed, void* dy, float* dw, float beta,
                            float* workspace, double* sums, void* stream);
/* Dropout keep bits of the K = 64 stage-1 Conv2D -> Dropout (-> BN) nodes
 * (resnet/wr_resnet.py:58-71's conv2a -> Dropout; the reference's Keras
 * Dropout mask, realised here by the pair-hash mask of acfe_dropout): the
 * forward writes one bit per output element, keep [N][H][W][K / 8] bytes (bit j
 * of byte (pixel, c / 8) = element (pixel, 8 (c / 8) + j) kept), and the BN-fold
 * weight gradient reads them instead of regenerating the mask -- identical
 * values.  _supported: the shapes (3x3 stride 1 "same", K = 64, C / 64 in
 * {1, 2, 4}, bf16) on which the forward can write them.  fwd_dropout_keep /
 * fwd_bn_keep = acfe_conv2d_fwd_dropout (pads 1, stats_partial required) /
 * acfe_conv2d_fwd_bn plus the keep output; wgrad_bnbwd_keep =
 * acfe_conv2d_wgrad_bnbwd (no residual `add`) with the mask from keep. */
int acfe_conv2d_dropout_keep_supported(int N, int H, int W, int C, int K, int dtype);
int acfe_conv2d_fwd_dropout_keep(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int pad_top,
                                 int pad_left, const float* bias, void* y, double* stats_partial, float drop_rate,
                                 unsigned long long seed, uint8_t* keep, void* stream);
int acfe_conv2d_fwd_bn_keep(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int pad_top,
                            int pad_left, const float* bias, void* y, double* stats_partial, float drop_rate,
                            unsigned long long seed, const float* bn_scale, const float* bn_shift, int bn_relu,
                            void* x_bn_out, uint8_t* keep, int dtype, void* stream);
int acfe_conv2d_wgrad_bnbwd_keep(const void* x, int N, int H, int W, int C, const void* gy, const void* u_bn, int K,
                                 const float* scale, const float* shift, int relu, const float* coef, float drop_rate,
                                 unsigned long long seed, const uint8_t* keep, void* dy, float* dw, float beta,
                                 float* workspace, double* sums, void* stream);

/* Stem convolution with one (folded) input channel and 16 outputs ("same",
 * stride 1, R = S = 5 (wr_resnet_bird) or 3 (wr_resnet)): the three identical
 * channels of tfdataset.py:2053 are folded by weff[r][s][k] = sum_c w[k][r][s][c]
 * (weff is tap-major, RSK, so one tap's 16 weights are contiguous). */
int acfe_stem_blocks(int N, int H, int W);
int acfe_stem_fold_weights(const float* w_krsc, int K, int R, int S, int C, float* weff, void* stream);
int acfe_stem_fwd(const void* x, int x_dtype, int N, int H, int W, int R, int S, int pad_top, int pad_left,
                  const float* weff, const float* bias, void* y, int y_dtype, double* stats_partial,
                  void* stream);
int acfe_stem_dgrad(const void* dy, int dy_dtype, int N, int H, int W, int R, int S, int pad_top,
                    int pad_left, const float* weff, void* dx, int dx_dtype, void* stream);
/* workspace: double[acfe_stem_blocks(N,H,W) * 16 * R * S]; dw is [16][R][S][rep]. */
int acfe_stem_wgrad(const void* x, int x_dtype, const void* dy, int dy_dtype, int N, int H, int W, int R,
                    int S, int pad_top, int pad_left, int rep, float* dw, float beta, double* workspace,
                    void* stream);
/* The stem backward with its BatchNormalization's backward apply folded in
 * (wr_resnet_bird.py:22-30: conv1_1 -> BN -> MaxPool2D((1, 2))): g = the BN
 * output gradient, xb = the BN input (the stem output), both bf16
 * [N][H][W][16] and 16-B aligned; coef = acfe_bn_bwd_finalize_ex's [3][16]
 * coefficients.  Writes dxin (bf16 [N][H][W]), dw (as acfe_stem_wgrad) and
 * bias_part double[acfe_stem_blocks(N,H,W)][2][16] (the conv-bias sums for
 * acfe_channel_sum_finalize) without storing dX_bn.  Replaces
 * acfe_bn_bwd_apply_ex + acfe_stem_dgrad + acfe_stem_wgrad + acfe_channel_sum
 * on that chain (the reference's autodiff of tf.keras Conv2D + BatchNormalization,
 * wr_resnet_bird.py:22-30). */
int acfe_stem_bwd_bn(const void* g, const void* xb, const void* xin, int N, int H, int W, int R, int S,
                     int pad_top, int pad_left, const float* weff, const float* scale, const float* shift,
                     const float* coef, int relu, void* dxin, int rep, float* dw, float beta,
                     double* bias_part, double* workspace, void* stream);

/* BatchNormalization(axis=3) (Keras: eps 1e-3, momentum 0.99, biased variance).
 * Partial slabs are double[acfe_reduce_blocks(rows)][2][C]. */
int acfe_reduce_blocks(long long rows);
int acfe_bn_stats(const void* x, long long rows, int C, int dtype, double* partial, void* stream);
int acfe_bn_finalize(const double* partial, int nrows, int ld, int C, double count, const float* gamma,
                     const float* beta, float eps, float momentum, float* moving_mean, float* moving_var,
                     int training, float* scale, float* shift, float* mean, float* invstd, void* stream);
int acfe_bn_apply(const void* x, int x_dtype, long long rows, int C, const float* scale, const float* shift,
                  int relu, void* y, int y_dtype, void* stream);
int acfe_bn_bwd_reduce(const void* dy, int dy_dtype, const void* x, int x_dtype, long long rows, int C,
                       const float* scale, const float* shift, const float* mean, const float* invstd,
                       int relu, double* partial, void* stream);
/* coef: float[3][C] for dx = a*g + b*x + c; dgamma/dbeta overwritten (nullable). */
int acfe_bn_bwd_finalize(const double* partial, int nrows, int C, double count, const float* scale,
                         const float* mean, const float* invstd, float* dgamma, float* dbeta, float* coef,
                         void* stream);
/* As acfe_bn_bwd_finalize; accumulate != 0 adds dgamma / dbeta into the given
 * buffers (a framework's gradient arena) instead of overwriting them. */
int acfe_bn_bwd_finalize_ex(const double* partial, int nrows, int C, double count, const float* scale,
                            const float* mean, const float* invstd, float* dgamma, float* dbeta, float* coef,
                            int accumulate, void* stream);
int acfe_bn_bwd_apply(const void* dy, int dy_dtype, const void* x, int x_dtype, long long rows, int C,
                      const float* scale, const float* shift, int relu, const float* coef, const void* add,
                      void* dx, int dx_dtype, void* stream);
/* acfe_bn_bwd_apply followed by the backward of the Dropout(rate, seed) whose
 * output was this BatchNormalization's input (no add). */
int acfe_bn_bwd_apply_dropout(const void* dy, int dy_dtype, const void* x, int x_dtype, long long rows, int C,
                              const float* scale, const float* shift, int relu, const float* coef,
                              float drop_rate, unsigned long long seed, void* dx, int dx_dtype, void* stream);
/* relu flags of acfe_bn_bwd_apply*: bit 0 = the BN's own ReLU (mask x*scale+shift > 0),
 * bit 1 = x itself is a ReLU output: dx (after the `add`) is multiplied by [x > 0],
 * the upstream ReLU's backward folded in. */
/* General form: residual `add` (nullable), Dropout backward (drop_rate > 0,
 * then add must be NULL), and per-channel sums of the stored dx into
 * sum_partial (nullable; slab [acfe_reduce_blocks(rows)][2][C] as
 * acfe_add_stats, its second (sum-of-squares) row left zero) -- the bias
 * gradient of the convolution whose output is this BatchNormalization's
 * input, via acfe_channel_sum_finalize. */
int acfe_bn_bwd_apply_ex(const void* dy, int dy_dtype, const void* x, int x_dtype, long long rows, int C,
                         const float* scale, const float* shift, int relu, const float* coef, const void* add,
                         float drop_rate, unsigned long long seed, void* dx, int dx_dtype, double* sum_partial,
                         void* stream);

/* Conv2D 3x3 "same" stride 1 -> MaxPool2D(2, 2) -> Dropout(rate, seed) with the
 * full-resolution conv output never stored (res{s}b0_branch21 -> pooling ->
 * dropout of resnet/wr_resnet_bird.py:139-148).  Supported shapes:
 * acfe_conv2d_pool_supported (bf16, C % 64 == 0, K in {64, 128}, W % 64 == 0,
 * H even).  acfe_conv2d_fwd_pool writes y [N][H/2][W/2][K], argmax bytes of the
 * same shape (first maximum, acfe_maxpool2d_fused's convention) and the BN
 * statistics slab of y (rows = acfe_conv2d_stats_rows(N*H*W, K), nullable).
 * The backward takes the gradient of the pooled, dropped-out values with the
 * dropout backward already applied (e.g. acfe_bn_bwd_apply_dropout):
 * acfe_conv2d_dgrad_unpool (wflip = acfe_conv2d_pack_weights(flip=1)) and
 * acfe_conv2d_wgrad_unpool (workspace as acfe_conv2d_wgrad, R = S = 3).
 * The row-halo kernels behind these entry points (and behind acfe_conv2d_fwd_add /
 * _fwd_bn / _fwd_add_bn / _fwd_pool_bn) store 16-byte runs: y / dx must be
 * 16-B aligned (ACFE_E_INVAL otherwise); acfe_conv2d_fwd / _dgrad fall back to
 * their generic kernels for a misaligned output. */
int acfe_conv2d_pool_supported(int N, int H, int W, int C, int K, int R, int S, int dtype);
int acfe_conv2d_fwd_pool(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int pad_top,
                         int pad_left, const float* bias, void* y, uint8_t* argmax, float drop_rate,
                         unsigned long long seed, double* stats_partial, int dtype, void* stream);
int acfe_conv2d_dgrad_unpool(const void* dy_pooled, const uint8_t* argmax, int N, int P, int Q, int K,
                             const void* wflip, int C, int pad_top, int pad_left, void* dx, int dtype, void* stream);
int acfe_conv2d_wgrad_unpool(const void* x, int N, int H, int W, int C, const void* dy_pooled, const uint8_t* argmax,
                             int K, int pad_top, int pad_left, float* dw, float beta, int dtype, float* workspace,
                             void* stream);

/* Conv2D 3x3 "same" stride 1 followed by the residual Add (+ReLU) of the block
 * (res{s}{b}_branch2b + Add, resnet/wr_resnet_bird.py:173-178): y = (ReLU)(conv(x)
 * + res), res/y [N][H][W][K] bf16, BN statistics of y into stats_partial (rows =
 * acfe_conv2d_stats_rows(N*H*W, K), nullable).  Shapes: acfe_conv2d_fwd_add_supported
 * (the rows kernel's, plus C % 8 == 0 / K % 128 == 0 bf16 layers -- the stage-2/3
 * conv2b -- on the generic kernel with the Add in its row stores; 16-B aligned
 * res / y there). */
int acfe_conv2d_rows_supported(int N, int H, int W, int C, int K, int R, int S, int dtype);
int acfe_conv2d_fwd_add_supported(int N, int H, int W, int C, int K, int dtype);
int acfe_conv2d_fwd_add(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int pad_top,
                        int pad_left, const float* bias, const void* res, int relu, void* y, double* stats_partial,
                        int dtype, void* stream);

/* BatchNormalization (+ReLU) prologue of the pre-activation blocks
 * (resnet/wr_resnet_bird.py:136-145 bn2a -> ReLU -> res{s}{b}_branch21,
 * :152-161 bn2b -> ReLU -> branch2b; the SURVEY §8b conv ABI's `bn_scale_shift`
 * argument): the conv reads the BN INPUT x and convolves x' = (ReLU)(x *
 * bn_scale[c] + bn_shift[c]) (acfe_bn_apply's values; zero padding applies to
 * x'), replacing acfe_bn_apply + the conv.  x' is written to x_bn_out
 * (nullable, [N][H][W][C] bf16) for the weight gradient.  bn_scale / bn_shift:
 * fp32 [C] from acfe_bn_finalize, 16-B aligned.  Shapes:
 * acfe_conv2d_bn_prologue_supported (3x3 stride-1 "same" bf16, C % 64 == 0,
 * C <= 256, K = 64).  acfe_conv2d_fwd_bn = acfe_conv2d_fwd_dropout (drop_rate
 * 0: none) with the prologue, acfe_conv2d_fwd_pool_bn = acfe_conv2d_fwd_pool
 * with it, acfe_conv2d_fwd_add_bn = acfe_conv2d_fwd_add with it. */
int acfe_conv2d_bn_prologue_supported(int N, int H, int W, int C, int K, int dtype);
int acfe_conv2d_fwd_bn(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int pad_top,
                       int pad_left, const float* bias, void* y, double* stats_partial, float drop_rate,
                       unsigned long long seed, const float* bn_scale, const float* bn_shift, int bn_relu,
                       void* x_bn_out, int dtype, void* stream);
int acfe_conv2d_fwd_pool_bn(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int pad_top,
                            int pad_left, const float* bias, void* y, uint8_t* argmax, float drop_rate,
                            unsigned long long seed, double* stats_partial, const float* bn_scale,
                            const float* bn_shift, int bn_relu, void* x_bn_out, int dtype, void* stream);
int acfe_conv2d_fwd_add_bn(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int pad_top,
                           int pad_left, const float* bias, const void* res, int relu, void* y, double* stats_partial,
                           const float* bn_scale, const float* bn_shift, int bn_relu, void* x_bn_out, int dtype,
                           void* stream);

/* Conv2D(1x1, 16 -> K in {64, 128}, bias) -> BatchNormalization -> (ReLU) as one
 * node whose conv output A = W x + b is never stored (csrc/c1bn.hip;
 * res{s}b0_branch2a0 + bn{s}b0_branch2a of resnet/wr_resnet_bird.py:121-131).
 * bf16 x [M][16] (16-B aligned), fp32 w [K][16] (KRSC, R = S = 1), bf16 y / dy
 * [M][K]; workspace float[acfe_c1bn_workspace(M, 16, K)].
 * Forward: acfe_c1bn_stats (training) writes partial = double[1][2][K] {sum A,
 * sum A^2} for acfe_bn_finalize(partial, 1, K, K, count = M, ...) and
 * gram = float[272] (sum x x^T, sum x; keep it for the backward; in eval mode
 * fill it with acfe_c1bn_stats too), then acfe_c1bn_apply writes y.
 * Backward: acfe_c1bn_bwd -> dx [M][16], dw [K][16], db [K], dgamma, dbeta
 * (nullable); count = M in training, 1e300 in eval.  The workspace also holds
 * the backward's fp32 [M][16] intermediate (W^T diag(scale)) g, so it grows
 * with M (64 B per pixel). */
int acfe_c1bn_supported(int C, int K);
long long acfe_c1bn_workspace(long long M, int C, int K);
int acfe_c1bn_stats(const void* x, long long M, int C, const float* w, int K, const float* bias, double* partial,
                    float* gram, float* workspace, void* stream);
int acfe_c1bn_apply(const void* x, long long M, int C, const float* w, int K, const float* bias, const float* scale,
                    const float* shift, int relu, void* y, void* stream);
int acfe_c1bn_bwd(const void* dy, const void* x, long long M, int C, const float* w, int K, const float* bias,
                  const float* scale, const float* shift, const float* mean, const float* invstd, int relu,
                  double count, const float* gram, void* dx, float* dw, float* db, float* dgamma, float* dbeta,
                  float* workspace, void* stream);
/* The three passes with a BatchNormalization (+ReLU) prologue on x (the
 * stride-2 block's bn2a0 -> ReLU in front of branch2a0, resnet/wr_resnet_bird.py
 * :121-127): x is the BN INPUT, every pass forms x' = (ReLU)(x * x_scale +
 * x_shift) (fp32 [16] from acfe_bn_finalize; acfe_bn_apply's values) and x' is
 * never stored; dx is the gradient for x'. */
int acfe_c1bn_stats_bn(const void* x, long long M, int C, const float* w, int K, const float* bias, double* part,
                       float* gram, float* workspace, const float* x_scale, const float* x_shift, int x_relu,
                       void* stream);
int acfe_c1bn_apply_bn(const void* x, long long M, int C, const float* w, int K, const float* bias,
                       const float* scale, const float* shift, int relu, void* y, const float* x_scale,
                       const float* x_shift, int x_relu, void* stream);
int acfe_c1bn_bwd_bn(const void* dy, const void* x, long long M, int C, const float* w, int K, const float* bias,
                     const float* scale, const float* shift, const float* mean, const float* invstd, int relu,
                     double count, const float* gram, void* dx, float* dw, float* db, float* dgamma, float* dbeta,
                     float* workspace, const float* x_scale, const float* x_shift, int x_relu, void* stream);

/* acfe_bn_bwd_apply_ex whose residual term is the backward of
 * AveragePooling2D(k, strides=k, "same") applied to x (the conv shortcut of the
 * stride-2 blocks): gpool = gradient of the pooled tensor [N][ceil(H/k)][ceil(W/k)][C]
 * (same dtype as dx), spread over each window's in-bounds elements. */
int acfe_bn_bwd_apply_pool(const void* dy, int dy_dtype, const void* x, int x_dtype, int N, int H, int W, int C,
                           const float* scale, const float* shift, int relu, const float* coef, const void* gpool,
                           int k, void* dx, int dx_dtype, double* sum_partial, void* stream);

/* acfe_bn_bwd_apply_ex whose residual term is the input gradient of a 1x1
 * "valid" Conv2D with stride k reading x (wr_resnet's transition-block
 * shortcut, resnet/wr_resnet.py:84-86, whose dX is nonzero only at the pixels
 * (k p, k q)): gsub = that gradient at those pixels, [N][(H-1)/k+1][(W-1)/k+1][C]
 * (same dtype as dx) -- the full-resolution shortcut gradient is never stored.
 * Bit-identical to acfe_bn_bwd_apply_ex with add = gsub scattered into zeros. */
int acfe_bn_bwd_apply_sub(const void* dy, int dy_dtype, const void* x, int x_dtype, int N, int H, int W, int C,
                          const float* scale, const float* shift, int relu, const float* coef, const void* gsub,
                          int k, void* dx, int dx_dtype, double* sum_partial, void* stream);

/* out[c] = beta*out[c] + sum_rows x[r][c] (bias gradients); partial as acfe_bn_stats. */
int acfe_channel_sum(const void* x, long long rows, int C, int dtype, double* partial, float* out, float beta,
                     void* stream);
/* out[c] = beta*out[c] + sum over the nrows slab rows of partial[r][0][c]. */
int acfe_channel_sum_finalize(const double* partial, int nrows, int C, float beta, float* out, void* stream);

/* Elementwise. */
int acfe_add(const void* a, const void* b, long long n, int relu, void* z, int dtype, void* stream);
/* z = a + b (+ReLU) over [rows][C] plus the BN statistics slab of z
 * (double[acfe_reduce_blocks(rows)][2][C]); C % 8 == 0 and 256 % (C/8) == 0. */
int acfe_add_stats(const void* a, const void* b, long long rows, int C, int relu, void* z, int dtype,
                   double* partial, void* stream);
int acfe_relu_bwd(const void* dy, const void* y, long long n, void* dx, int dtype, void* stream);
/* acfe_relu_bwd over [rows][C] plus per-channel sums of dx (slab as acfe_add_stats). */
int acfe_relu_bwd_sum(const void* dy, const void* y, long long rows, int C, void* dx, int dtype, double* partial,
                      void* stream);
int acfe_dropout(const void* x, long long n, float rate, unsigned long long seed, void* y, int dtype,
                 void* stream);
int acfe_cast(const void* x, int x_dtype, long long n, void* y, int y_dtype, void* stream);
int acfe_sigmoid(const float* z, long long n, float* p, void* stream);

/* Pooling (NHWC). MaxPool2D valid (gradient to the first maximum);
 * AveragePooling2D "same" with strides == pool (in-bounds averaging). */
int acfe_maxpool2d(const void* x, int N, int H, int W, int C, int kh, int kw, void* y, int dtype,
                   void* stream);
int acfe_maxpool2d_bwd(const void* x, const void* dy, int N, int H, int W, int C, int kh, int kw, void* dx,
                       int dtype, void* stream);
/* MaxPool2D (kh,kw) in {(1,2),(2,2),(3,3)} -> optional Dropout(rate, seed) ->
 * optional BN statistics slab (partial, as acfe_add_stats; may be NULL), and the
 * argmax byte of every output element (first maximum, may be NULL; 8-B aligned). */
int acfe_maxpool2d_fused(const void* x, int N, int H, int W, int C, int kh, int kw, void* y, uint8_t* argmax,
                         float drop_rate, unsigned long long seed, double* partial, int dtype, void* stream);
/* MaxPool2D((kh, kw)) of BatchNormalization(x) (+ReLU) with y = x * scale[c] +
 * shift[c] formed at load time and rounded to the storage type, exactly the
 * values acfe_bn_apply would store; argmax bytes and BN statistics of the
 * pooled output as acfe_maxpool2d_fused (no dropout).  Replaces the
 * BatchNormalization -> MaxPool2D((1, 2)) pair of wr_resnet_bird.py:29-30. */
int acfe_bn_maxpool2d_fused(const void* x, int N, int H, int W, int C, const float* scale, const float* shift,
                            int relu, int kh, int kw, void* y, uint8_t* argmax, double* stats_part, int dtype,
                            void* stream);
/* Backward of acfe_maxpool2d_fused from its argmax bytes (x is not re-read). */
int acfe_maxpool2d_bwd_argmax(const uint8_t* argmax, const void* dy, int N, int H, int W, int C, int kh, int kw,
                              float drop_rate, unsigned long long seed, void* dx, int dtype, void* stream);
/* acfe_maxpool2d_bwd_argmax (no dropout) fused with the acfe_bn_bwd_reduce of
 * the BatchNormalization in front of the pool (wr_resnet_bird.py:29-30, the
 * stem's BN -> MaxPool2D((1, 2)); backward of acfe_bn_maxpool2d_fused): the
 * expanded gradient dx is written and, with x = the BN input, the reduce slab
 * part [acfe_reduce_blocks(N*H*W)][2][C] = {sum g, sum g * (x - mean) * invstd}
 * (g = dx masked by the BN's ReLU when relu) for acfe_bn_bwd_finalize_ex. */
int acfe_maxpool2d_bwd_argmax_bn(const uint8_t* argmax, const void* dy, int N, int H, int W, int C, int kh, int kw,
                                 void* dx, int dtype, const void* x, const float* scale, const float* shift,
                                 const float* mean, const float* invstd, int relu, double* part, void* stream);
int acfe_avgpool2d(const void* x, int N, int H, int W, int C, int k, void* y, int dtype, void* stream);
int acfe_avgpool2d_bwd(const void* dy, int N, int H, int W, int C, int k, void* dx, int dtype, void* stream);
/* Reduce the middle axis of [outer][L][inner] to fp32 [outer][inner]:
 * mode 0 = log-mean-exp with sharpness (wr_resnet_bird.py:83-87), 1 = mean. */
int acfe_axis_pool(const void* x, int x_dtype, long long outer, int L, int inner, float sharpness, int mode,
                   float* y, void* stream);
int acfe_axis_pool_bwd(const void* x, int x_dtype, const float* dy, long long outer, int L, int inner,
                       float sharpness, int mode, void* dx, void* stream);

/* Dense (Keras kernel layout [in][out]) and losses on its sigmoid output:
 * mode 0 BinaryCrossentropy, 1 CategoricalCrossentropy (audiomodel.py:1206-1223).
 * workspace: float[B]. */
int acfe_dense_fwd(const float* x, const float* w, const float* bias, int B, int I, int O, float* z,
                   void* stream);
int acfe_dense_bwd(const float* x, const float* w, const float* dz, int B, int I, int O, float* dx, float* dw,
                   float* db, void* stream);
int acfe_loss(const float* z, const float* y, int B, int L, int mode, float grad_scale, float* loss, float* dz,
              float* workspace, void* stream);

/* Adam (tf.keras.optimizers.Adam, audiomodel.py:1226-1240) over a flat fp32
 * parameter arena; alpha = lr*sqrt(1-b2^t)/(1-b1^t). */
int acfe_adam_step(float* params, const float* grads, float* m, float* v, long long n, float grad_scale,
                   float beta1, float beta2, float eps, float alpha, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ACFE_H */
