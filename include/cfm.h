/* cfm.h — C ABI of the MI355X-native Conformer encoder hot path (libcfm.so).
 *
 * Plain C: raw device pointers, sizes and a hipStream_t passed as void*.  No torch types.
 * Every entry point is stream-ordered (no host synchronisation), allocates no device memory
 * (callers pass workspaces), keeps no pointer after return, and returns 0 on success or a
 * negative CFM_ERR_* code; cfm_get_last_error() returns the thread's last message.
 *
 * The reference (icadriani/nn_conformer_for_speech_recognition) has no FFI: its hot path is a
 * composition of torch.nn modules.  Each entry point below names the reference module/op it
 * replaces (file:line under /root/reference, or torchaudio semantics restated in
 * oracle/conformer.py); INTEGRATION.md shows the ctypes binding the host side uses.
 *
 * Layouts: activations are token-major (row = b*T + t, feature contiguous), matching
 * torchaudio's (B, T, D) interface after its internal transpose.  dtype codes: CFM_F32 / CFM_BF16.
 */
#ifndef CFM_H
#define CFM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CFM_F32 0
#define CFM_BF16 1
#define CFM_FP8 2   /* OCP e4m3fn (gfx950), GEMM operands only (cfm_gemm, cfm_quant_fp8) */

#define CFM_OK 0
#define CFM_ERR_ARG (-1)
#define CFM_ERR_SHAPE (-2)
#define CFM_ERR_DTYPE (-3)
#define CFM_ERR_ALIGN (-4)
#define CFM_ERR_UNSUPPORTED (-5)
#define CFM_ERR_LAUNCH (-6)

#define CFM_ACT_NONE 0
#define CFM_ACT_SILU 1

int cfm_version(void);
const char* cfm_get_last_error(void);

/* Graph-safe dropout streams.  Binds a DEVICE uint64 step counter for this process (nullptr
   unbinds).  While bound, every dropout-capable kernel (GEMM epilogue, scale_dropout, attention)
   reads the counter when it RUNS and uses seed + counter * 0x9E3779B97F4A7C15 instead of the
   seed passed at launch, so a training step captured once into a HIP graph draws fresh masks on
   every replay after the caller increments the counter on the stream.  Backward kernels see the
   same counter value as their forward within a step, so masks regenerate bit-identically.
   Replaces the per-call torch RNG state of nn.Dropout (asrnn.py:31, torchaudio Conformer). */
int cfm_rng_bind(const uint64_t* counter);

/* Measurement probes (bench.py roofline timing, also inside a captured HIP graph where HIP events
   cannot be read back on ROCm).  A probe slot is 4 x u64 {start, end, total, count}: mode 0
   resets start = ~0, end = 0 (before the probed launch, which records its first-start / last-end
   into start / end, see cfm_gemm_desc.probe); mode 1 adds end - start to total and 1 to count
   (after it).  Modes 2 / 3 take an 8 x u64 slot {start, end, total, count, stamp, total_incl, -, -}:
   mode 2 is mode 0 plus stamp = the wall clock when this one-lane kernel runs, mode 3 is mode 1 plus
   total_incl += (the wall clock when this one-lane kernel runs) - stamp: stamp-to-stamp around the
   probed launch.  Minus the same interval of an EMPTY pair (mode 2 directly followed by mode 3:
   the two one-lane kernels' own dispatch), it is the time the launch adds to a serial stream --
   its dispatch ramp, execution and end-of-kernel completion, what rocprofv3's kernel trace counts.
   Ticks of the constant-rate GPU wall clock at cfm_wallclock_khz() kHz. */
int cfm_probe_slot(unsigned long long* slot, int mode, void* stream);
int cfm_wallclock_khz(void);

/* y[i] = (dy)x[i] for n elements (dtype conversion; fp32 master weights -> bf16 compute copies). */
int cfm_cast(const void* x, int dtype_x, void* y, int dtype_y, long n, void* stream);

/* Many casts in one launch (the per-step bf16 shadow of every weight matrix): `tasks` is a
   DEVICE array of ntasks cfm_cast_task; task t owns blocks [blk0, blk0 + ceil(n / 2048)) of a grid of
   `nblocks` blocks (blk0 ascending, tasks back to back).  Replaces one cfm_cast launch per weight. */
typedef struct {
  const void* src;
  void* dst;
  long n;
  long blk0;
} cfm_cast_task;
int cfm_cast_batch(const cfm_cast_task* tasks, int ntasks, long nblocks, int dtype_x, int dtype_y,
                   void* stream);

/* Transposed casts in one launch: dst (cols x rows) = (dy) src (rows x cols)^T, row-major both,
   and (when dst_n != NULL) the plain copy dst_n (rows x cols) = (dy) src from the same read.
   Task t owns blocks [blk0, blk0 + ceil(rows/64) * ceil(cols/64)) (64 x 64 tiles).  Used for the
   per-step K-major bf16 copies W^T of the weight matrices, so the data-gradient GEMMs dX = dY W
   read both operands K-major (replaces the MN-major B path of those GEMMs; no reference
   counterpart -- autograd's mm backward, torch/csrc/autograd/FunctionsManual.cpp mm_mat1_backward). */
typedef struct {
  const void* src;   /* fp32 */
  void* dst;         /* transposed copy */
  void* dst_n;       /* optional row-major copy (NULL: none) */
  long rows, cols;
  long blk0;
} cfm_castT_task;
int cfm_cast_transpose_batch(const cfm_castT_task* tasks, int ntasks, long nblocks, int dtype_x, int dtype_y,
                             void* stream);

/* ---------------------------------------------------------------- SpecAugment
 * Replaces ASRNN.SpecAugment / time_warping / frequency_masking / time_masking
 * (lib/standard/asrnn.py:91-192).  The random draws stay on the host (python `random`, the
 * reference's own RNG, in the reference's order); this kernel applies them in ONE pass:
 * y[b,f,t] = x[b,f,Wt_b(t)] (warp passes composed), then the masks when intended != 0
 * (the reference's masks are no-ops as shipped, asrnn.py:141,165).
 * params (device int32): [n_warp, n_freq, n_time, 0,
 *                         n_warp x B x (w, w0, tau), n_freq x (f0, f), n_time x B x (t0, t)]
 * x, y: (B, F, T) fp32, may not alias. */
int cfm_specaug_apply(const float* x, float* y, int B, int F, int T, const int32_t* params,
                      int n_params, int intended, float mask_value, void* stream);

/* ---------------------------------------------------------------- log-mel front-end
 * Replaces the CPU feature step of lib/standard/speechcommands.py:113-119:
 * librosa.feature.melspectrogram(y, sr, n_mels) (periodic Hann, center=True zero padding, |rfft|^2,
 * Slaney mel bank) -> np.where(mel < 1e-10, 0, log(mel)) -> per-utterance min-max (normalize != 0),
 * frames past 1 + lens[b] / hop zero (the collate's padding, speechcommands.py:188).
 * wave (B, ld_wave) fp32, lens (B,) int32 samples; n_fft a power of two in [16, 4096];
 * window (n_fft,) fp32; twiddle (n_fft/2) complex fp32 pairs exp(-2 pi i k / n_fft);
 * filter m = mel_w[mel_off[m] ...+ mel_cnt[m]) applied to power bins mel_lo[m] ...;
 * out (B, n_mels, nT) fp32; ws >= cfm_logmel_ws_bytes(B, nT). */
size_t cfm_logmel_ws_bytes(int B, int nT);
int cfm_logmel_fwd(const float* wave, long ld_wave, const int32_t* lens, int B, int n_fft, int hop,
                   const float* window, const float* twiddle, const int32_t* mel_lo, const int32_t* mel_cnt,
                   const int32_t* mel_off, const float* mel_w, int n_mels, int nT, int normalize, float* out,
                   float* ws, void* stream);

/* ---------------------------------------------------------------- GEMM (MFMA)
 * C[z][m][n] = epilogue( alpha * sum_k A(m,k) * B(n,k) )  for z in [0, batch).
 * Serves every dense contraction of the encoder (torch.nn.Linear / 1x1 Conv1d forward,
 * input-grad and weight-grad): FFN (torchaudio _FeedForwardModule), MHSA in/out projections
 * (nn.MultiheadAttention), point-wise convs (_ConvolutionModule), the front-end projection
 * (asrnn.py:208 / frame projection) and the projection block (asrnn.py:73-89).
 *   A(m,k) = A[m*lda + k] if a_kmajor else A[k*lda + m]
 *   B(n,k) = B[n*ldb + k] if b_kmajor else B[k*ldb + n]
 * (A / B rows may overlap, ld below the row length, only with allow_overlap: read-only windowed views,
 *  cfm_ffold_*.)
 * Epilogue, in order: v = alpha*acc + bias[n];  v *= act'(pre[m,n]) if act_grad;
 *   if act == SILU { pre[m,n] = v (if pre != NULL); v = silu(v) };  v *= dropout(seed, idx);
 *   v *= out_scale;  v += residual[m,n];  C = v  (or atomically C += v when split_k > 1).
 * dtype_ab is the operand type (fp32 operands run on the exact-f32 MFMA path). */
typedef struct cfm_gemm_desc {
  int M, N, K, batch;
  int dtype_ab;
  const void* A; long lda; long stride_a; int a_kmajor;
  const void* B; long ldb; long stride_b; int b_kmajor;
  void* C; long ldc; long stride_c; int dtype_c;
  float alpha;
  const float* bias;
  int act;                 /* CFM_ACT_NONE | CFM_ACT_SILU */
  int act_grad;            /* multiply by silu'(pre) (backward of a SILU epilogue) */
  void* pre; int dtype_pre;
  float drop_p; uint64_t drop_seed; uint64_t drop_offset;
  float out_scale;
  const void* residual; long ldr; int dtype_r;
  int split_k;             /* >1: C must be fp32 with a plain epilogue (alpha, bias) */
  float* workspace;        /* split_k > 1: NULL -> partial sums are atomically added into a
                              pre-initialised C; else >= split_k*batch*M*N floats of slabs that a
                              second pass reduces into C (deterministic, no pre-initialisation) */
  unsigned long long* probe; /* optional timing slot (measurement only): the launch atomically
                              min-records its first workgroup's start and max-records its last
                              workgroup's end (s_memrealtime ticks) into probe[0] / probe[1] */
  float* a_colsum;         /* optional (bf16 LDS-DMA path, MN-major A, split_k > 1 with workspace, batch 1):
                              a_colsum[m] = sum_k A(m, k) -- the bias gradient of a weight-gradient GEMM
                              dW = dY^T X (A = dY^T) -- from the staged A tiles; workspace then needs
                              split_k*M more floats.  NULL: off. */
  const void* rowdot_with; /* optional (bf16 C, LDS-DMA path, N % 64 == 0, batch 1, no split): per row m = b*T + t and
                              64-column group g, rowdot_out[(b * N/64 + g) * T + t] = sum_n C[m][n] * rowdot_with[m*ldc + n]
                              over the bf16-rounded C -- attention's D = rowsum(dO * O) per head (dk = 64) from the
                              out-projection data-gradient GEMM that produces dO.  NULL: off. */
  float* rowdot_out;
  int rowdot_T;
  /* dtype_ab == CFM_FP8: device scalars multiplied into alpha (the per-tensor dequantisation scales
     written by cfm_quant_fp8); NULL: 1 */
  const float* alpha_a_dev;
  const float* alpha_b_dev;
  /* nonzero: A / B rows may overlap (lda / ldb below the row length: the folded front-end's read-only windowed
     view of the packed mels, cfm_ffold_*).  0: lda >= (a_kmajor ? K : M) and ldb >= (b_kmajor ? K : N) are
     enforced (CFM_ERR_SHAPE), so a wrongly transposed view fails instead of reading overlapping rows. */
  int allow_overlap;
  /* dtype_ab == CFM_FP8 with MX operands (both or neither): the e8m0 block scales of A and B as cfm_quant_mx
     writes them ([M][K/32] / [N][K/32] bytes, one per 32 consecutive K elements of a row); the block-scaled MFMA
     applies them per 32-element run (alpha_*_dev must be NULL).  K % 128 == 0, K <= 2048. */
  const uint8_t* mx_a;
  const uint8_t* mx_b;
  /* optional second output (MX fp8 launches with the FFN-up epilogue -- bias + SiLU + bf16 pre + dropout, bf16 C,
     ldc == N, N % 32 == 0): the MX e4m3 copy of the bf16 C, exactly cfm_quant_mx of it -- mx_out (M x N e4m3),
     mx_out_scales (M x N/32 e8m0) -- the next fp8 GEMM's operand, written by the same epilogue.  NULL: off. */
  void* mx_out;
  uint8_t* mx_out_scales;
} cfm_gemm_desc;
int cfm_gemm(const cfm_gemm_desc* d, void* stream);
/* Per-tensor fp8 (e4m3fn) quantisation for the fp8 GEMM path (configs[4]; no reference counterpart -- the
   reference computes in fp32): y = e4m3(x * 2^k), k the largest with amax(|x|) * 2^k <= 448, *inv_scale = 2^-k (device scalar for
   cfm_gemm_desc.alpha_*_dev); amax_ws: cfm_quant_fp8_ws_bytes() of scratch.  x fp32 or bf16, 16-B aligned. */
size_t cfm_quant_fp8_ws_bytes(void);
int cfm_quant_fp8(const void* x, int dtype_x, long n, void* y, float* inv_scale, unsigned* amax_ws, void* stream);
/* Batched cfm_quant_fp8 over a device table of tensors (the per-step fp8 copies of a model's forward GEMM
   weights, configs[4]): TWO launches for the whole list instead of two per tensor; per tensor the same
   current scaling, scale and e4m3 bytes as cfm_quant_fp8 (the max is order-independent: bit-identical).
   Replaces the per-weight quantisation loop of the fp8 path (no reference counterpart: the reference has
   no fp8).  tasks: device array; blk0 = prefix sum of cfm_quant_fp8_batch_blocks(n) over the tasks;
   amax_ws: nblocks floats of scratch. */
typedef struct {
  const void* x;      /* fp32 or bf16 (dtype_x of the call), 16-B aligned */
  void* y;            /* e4m3 bytes, 8-B aligned */
  float* inv_scale;   /* dequantisation factor 2^-k (device scalar) */
  long n;
  long blk0;
} cfm_q8_task;
long cfm_quant_fp8_batch_blocks(long n);
int cfm_quant_fp8_batch(const cfm_q8_task* tasks, int ntasks, long nblocks, int dtype_x, float* amax_ws,
                        void* stream);
/* y = float(x) * inv_scale (inv_scale NULL: 1) -- the dequantised view, for tests. */
int cfm_dequant_fp8(const void* x, long n, const float* inv_scale, float* y, void* stream);
/* MX e4m3 quantisation (OCP microscaling; configs[4]'s fp8 path, no reference counterpart): every 32
   consecutive elements of a row share one e8m0 scale byte s = 127 - k, k the largest integer with
   amax(block) * 2^k <= 448 (0 for an all-zero block), and y = e4m3(x * 2^k) (round to nearest even).
   x: rows x K (row stride ldx elements, fp32 or bf16, 16-B aligned), K % 32 == 0; y: rows x K bytes
   (row stride K); s: rows x K/32 bytes (row-major).  One pass, no tensor-wide amax: the operand form of
   cfm_gemm_desc.mx_a / mx_b. */
int cfm_quant_mx(const void* x, int dtype_x, long rows, int K, long ldx, void* y, uint8_t* s, void* stream);
/* Batched cfm_quant_mx over a device table (the per-step MX copies of the forward GEMM weights): ONE launch;
   blk0 = prefix sum of cfm_quant_mx_batch_blocks(rows, K); rows of each tensor contiguous (ldx = K). */
typedef struct {
  const void* x;      /* fp32 or bf16 (dtype_x of the call), 16-B aligned */
  void* y;            /* e4m3 bytes, 8-B aligned */
  uint8_t* s;         /* e8m0 block scales, rows x K/32 */
  long rows;
  int K;
  int pad;
  long blk0;
} cfm_mx_task;
long cfm_quant_mx_batch_blocks(long rows, int K);
int cfm_quant_mx_batch(const cfm_mx_task* tasks, int ntasks, long nblocks, int dtype_x, void* stream);
/* y[i] = e4m3(x[i]) * 2^(s[i / 32] - 127) -- the dequantised view of an MX tensor (n % 32 == 0), for tests. */
int cfm_dequant_mx(const void* x, const uint8_t* s, long n, float* y, void* stream);
/* Grouped weight gradients: every dW_i (N_i x K_i, fp32) = dY_i^T X_i over the same M tokens (dY_i (M x N_i),
   X_i (M x K_i) bf16 row-major) and optionally db_i = sum_rows dY_i, in ONE launch of 256x128 tiles that each
   run the whole token reduction (no split-K).  The caller fills a HOST table (cfm_wgrad_group_fill, one
   entry of cfm_wgrad_group_task_bytes() per GEMM, tile0 = running sum of cfm_wgrad_group_tiles), copies it
   to the device and launches total_tiles workgroups.  Replaces the per-GEMM split-K weight gradients of
   the encoder backward (torch autograd's per-Linear mm for grad_weight, FunctionsManual.cpp). */
size_t cfm_wgrad_group_task_bytes(void);
long cfm_wgrad_group_tiles(int N, int K);
int cfm_wgrad_group_fill(void* host_table, int i, const void* dy, const void* x, float* dw, float* db, int M,
                         int N, int K, long tile0);
int cfm_wgrad_group(const void* dev_table, int ntasks, long total_tiles, void* stream);
/* Grouped deterministic column reductions: the small deferred reductions of a backward pass (LayerNorm
   dgamma|dbeta partial rows -- torch's LayerNorm backward weight/bias sums --, depthwise-conv weight/bias
   partials) in ONE launch.  Host table of cfm_colreduce_group_task_bytes() per task (block0 = running sum of
   cfm_colreduce_group_blocks(N)); mode 0: out[n] = sum_p part[p*ldp + n]; mode 1: the depthwise-conv
   [K+1][C] sums scattered to dw (C x K) and db (C). */
size_t cfm_colreduce_group_task_bytes(void);
long cfm_colreduce_group_blocks(long N);
int cfm_colreduce_group_fill(void* host_table, int i, const float* part, int nparts, long N, long ldp, float* out,
                             float* out2, int mode, int C, int K, long block0);
int cfm_colreduce_group(const void* dev_table, int ntasks, long total_blocks, void* stream);
/* the same launch with a timing slot (as cfm_gemm_desc.probe: first-workgroup start / last-workgroup end) */
int cfm_wgrad_group_probed(const void* dev_table, int ntasks, long total_tiles, unsigned long long* probe,
                           void* stream);
/* Planned grouped weight gradients (the encoder backward's default): cfm_wgrad_group_plan packs the tasks'
   tiles (task_tiles[i] = cfm_wgrad_group_tiles(N_i, K_i)) into rounds of one tile per CU per XCD (nxcd XCDs of
   cus CUs) made of whole tasks -- the tiles sharing a dY or X column slice co-resident on one XCD, which then
   streams the slice through its L2 once -- and splits the tiles of the ragged last round over K slices
   (task_split[i] > 1), so that round fills the chip.  It writes one schedule word per workgroup (sched, capacity
   cap) and returns the grid size (< 0: error).  Fill the table with cfm_wgrad_group_fill_split (split = the
   plan's task_split[i]; ws = cfm_wgrad_group_ws_floats(N, K, split) floats of fp32 workspace for a split task;
   red0 = running sum of cfm_wgrad_group_red_blocks), copy table and schedule to the device and launch
   cfm_wgrad_group_sched (red_blocks = the total): the GEMM launch, then the deterministic slab reduction of the
   split tasks into dw / db.  probe: optional timing slot (as cfm_wgrad_group_probed). */
long cfm_wgrad_group_plan(const long* task_tiles, int ntasks, int nxcd, int cus, unsigned* sched, long cap,
                          int* task_split);
long cfm_wgrad_group_ws_floats(int N, int K, int split);
long cfm_wgrad_group_red_blocks(int N, int K, int split);
int cfm_wgrad_group_fill_split(void* host_table, int i, const void* dy, const void* x, float* dw, float* db, int M,
                               int N, int K, int split, float* ws, long red0);
int cfm_wgrad_group_sched(const void* dev_table, int ntasks, const unsigned* dev_sched, long grid, long red_blocks,
                          unsigned long long* probe, void* stream);
/* kernel-selection switch for A/B measurements: bit 0 = 256-row register-staged tiles allowed,
   bit 1 = LDS-DMA pipelined kernel allowed, bit 3 = timing experiment (pipelined kernels skip their
   stores), bits 4-6 = pipelined variant (0 auto, 1 256x128/BK64, 2 256x128/BK32 two per CU,
   5 192x128, 7 192x128/BK32 two per CU), bit 10 = generic dropout hash path, bit 12 = no 192-row rule for
   1024/1536-wide outputs, bit 13 = timing experiment (main loop skipped: epilogue only), bit 14 = generic
   epilogue rows instead of the compile-time epilogue kinds, bit 19 = shared-DMA pipeline instead of the
   warp-specialised kernel for d-wide outputs, bit 21 = 192-row pipeline instead of the warp-specialised kernel
   for 1024/1536-wide outputs; default 3. */
int cfm_gemm_set_mode(int mode);

/* out[n] (+)= sum_m x[m*ld + n]  — bias gradients (sum over tokens).  ws: >= 4*N*256 bytes. */
/* out[n] (+)= sum_p part[p * ldp + n] for n < N: the deterministic second level of every partial-row
   reduction (LayerNorm dgamma|dbeta partials left by cfm_layernorm_bwd with NULL dgamma/dbeta, so the
   weight-gradient reduction can run on another stream). */
int cfm_colreduce(const float* part, int nparts, long N, long ldp, float* out, int accumulate, void* stream);
int cfm_colsum(const void* x, int dtype_x, long M, int N, long ld, float* out, int accumulate,
               float* ws, void* stream);

/* ---------------------------------------------------------------- LayerNorm (nn.LayerNorm(D))
 * Forward: y = (x-mean)*rstd*gamma + beta; saves mean/rstd per row.
 * Backward: dx = rstd*(g - mean(g) - xhat*mean(g*xhat)) + dres, g = dy*gamma;
 * dgamma/dbeta accumulate (+=) over rows.  ws: >= 8*D*nblk bytes, see cfm_layernorm_ws_bytes. */
int cfm_layernorm_fwd(const void* x, int dtype_x, const float* gamma, const float* beta, void* y,
                      int dtype_y, float* mean, float* rstd, long M, int D, float eps, void* stream);
/* The same forward (fp32 x, bf16 y) with a second output: y's MX e4m3 copy -- y8 (M x D e4m3) and s8
   (M x D/32 e8m0), exactly cfm_quant_mx of the bf16 y -- for the fp8 forward GEMM that consumes it
   (configs[4]); D in {256, 512, 1024}. */
int cfm_layernorm_fwd_mx(const float* x, const float* gamma, const float* beta, void* y, void* y8, uint8_t* s8,
                         float* mean, float* rstd, long M, int D, float eps, void* stream);
/* The same with x of dtype_x (CFM_F32 or CFM_BF16: the bf16 mode's bf16 residual stream). */
int cfm_layernorm_fwd_mx_ex(const void* x, int dtype_x, const float* gamma, const float* beta, void* y, void* y8,
                            uint8_t* s8, float* mean, float* rstd, long M, int D, float eps, void* stream);
/* The residual add of the module before a LayerNorm, done by the LayerNorm: xout = x + delta (fp32; delta of dtype_d,
   CFM_BF16 -- the module's GEMM output with bias, dropout and out_scale, no residual -- or CFM_F32), then
   y = LN(xout) as cfm_layernorm_fwd, and, with y8 / s8 non-null, y's MX copy as cfm_layernorm_fwd_mx.  Replaces the
   residual-stream GEMM epilogue `x + out_scale * dropout(h W^T + b)` (torchaudio ConformerLayer, ffn / attention /
   conv residual adds; asrnn.py:214) followed by the next module's LayerNorm.  xout must not alias x or
   delta. */
int cfm_layernorm_fwd_res(const float* x, const void* delta, int dtype_d, float* xout, const float* gamma,
                          const float* beta, void* y, int dtype_y, void* y8, uint8_t* s8, float* mean, float* rstd,
                          long M, int D, float eps, void* stream);
size_t cfm_layernorm_ws_bytes(long M, int D);
int cfm_layernorm_bwd(const void* dy, int dtype_dy, const void* x, int dtype_x, const float* gamma,
                      const float* mean, const float* rstd, const void* dres, int dtype_dres,
                      void* dx, int dtype_dx, float* dgamma, float* dbeta, float* ws, long M, int D,
                      void* stream);
/* The same plus g2 (bf16, M x D) = dx * g2_scale * dropout(g2_p, g2_seed, element index) -- exactly
   cfm_scale_dropout(dx, ..., offset 0) -- written by the same pass: the next module's (residual-
   dropout) input gradient in the encoder backward.  g2 == NULL: identical to cfm_layernorm_bwd. */
int cfm_layernorm_bwd_drop(const void* dy, int dtdy, const void* x, int dtx, const float* gamma,
                           const float* mean, const float* rstd, const void* dres, int dtres, void* dx,
                           int dtdx, float* dgamma, float* dbeta, float* ws, long M, int D, void* g2,
                           float g2_scale, float g2_p, uint64_t g2_seed, void* stream);

/* y = act(x*scale [dropout]) + residual, elementwise helpers used at residual joins. */
int cfm_scale_dropout(const void* x, int dtype_x, void* y, int dtype_y, long n, float scale,
                      float drop_p, uint64_t seed, uint64_t offset, void* stream);

/* dx = dy * silu'(pre) elementwise (backward of a SILU GEMM epilogue when the gradient feeds a
 * weight-gradient GEMM directly, e.g. the projection block asrnn.py:84-87). */
int cfm_silu_bwd(const void* dy, int dtype_dy, const void* pre, int dtype_pre, void* dx, int dtype_dx,
                 long n, void* stream);

/* ---------------------------------------------------------------- Convolution module
 * _ConvolutionModule (torchaudio; restated oracle/conformer.py ConvModuleRef):
 *   a = pw1(LN(x)) (cfm_gemm), g = GLU(a) (dim = channel), y = depthwise_conv_K(g) + b,
 *   z = SiLU(BatchNorm1d(y)) (train: batch statistics over B*T incl. padded frames),
 *   out = pw2(z) (cfm_gemm, + residual).
 * a: (B*T, 2C) token-major; w_dw: (C, K) fp32; y: (B*T, C) fp32.
 * cfm_glu_dwconv_fwd also produces per-channel partial (sum, sumsq) into ws for BN. */
size_t cfm_convmod_ws_bytes(int B, int T, int C, int K);
/* rows of cfm_glu_dwconv_bwd's [nparts][K+1][C] weight-gradient partials in ws (mode 1 of cfm_colreduce_group) */
long cfm_convmod_nparts(int B, int T);
int cfm_glu_dwconv_fwd(const void* a, int dtype_a, const float* w_dw, const float* b_dw, float* y,
                       int B, int T, int C, int K, float* ws, void* stream);
/* z = silu(bn(y)).  training: batch stats finalised from the partial sums cfm_glu_dwconv_fwd left
 * in ws (same B, T, C), running stats updated (momentum, unbiased var); eval: running stats.
 * Writes mean/invstd (C each) for the backward. */
int cfm_bn_silu_fwd(const float* y, const float* gamma, const float* beta, float* running_mean,
                    float* running_var, float momentum, float eps, int training, float* mean,
                    float* invstd, void* z, int dtype_z, int B, int T, int C, const float* ws,
                    void* stream);
/* backward of z = silu(bn(y)): dy = BN-bwd(dz*silu'(bn(y))); dgamma, dbeta (=) written. */
int cfm_bn_silu_bwd(const void* dz, int dtype_dz, const float* y, const float* gamma,
                    const float* beta, const float* mean, const float* invstd, int training,
                    float* dy, float* dgamma, float* dbeta, long M, int C, float* ws, void* stream);
/* SyncBatchNorm split of cfm_bn_silu_fwd / cfm_bn_silu_bwd (the host all-reduces `sums` / the dbeta|dgamma
   sums between the halves; M_total = rows over all replicas).  Replaces torch.nn.SyncBatchNorm over the
   ConvModule's BatchNorm1d (torchaudio conformer, asrnn.py:29) under data parallelism. */
int cfm_bn_silu_fwd_sums(const float* ws, int B, int T, int C, float* sums, void* stream);
int cfm_bn_silu_fwd_apply(const float* y, const float* gamma, const float* beta, float* running_mean,
                          float* running_var, float momentum, float eps, const float* sums, long M_total, float* mean,
                          float* invstd, void* z, int dtz, long M, int C, void* stream);
int cfm_bn_silu_bwd_sums(const void* dz, int dtdz, const float* y, const float* gamma, const float* beta,
                         const float* mean, const float* invstd, long M, int C, float* ws, float* dbeta, float* dgamma,
                         void* stream);
int cfm_bn_silu_bwd_apply(const void* dz, int dtdz, const float* y, const float* gamma, const float* beta,
                          const float* mean, const float* invstd, const float* dbeta_total, const float* dgamma_total,
                          long M_total, float* dy, long M, int C, void* stream);
/* Generic BatchNorm1d over (M, C) rows with optional SiLU after the normalisation (act = 1) —
 * the projection block's BatchNorm1d(256) (lib/standard/asrnn.py:32,88).  ws: cfm_bn_ws_bytes(C). */
size_t cfm_bn_ws_bytes(int C);
int cfm_bn_fwd(const float* y, const float* gamma, const float* beta, float* running_mean,
               float* running_var, float momentum, float eps, int training, float* mean, float* invstd,
               void* z, int dtype_z, long M, int C, int act, float* ws, void* stream);
int cfm_bn_bwd(const void* dz, int dtype_dz, const float* y, const float* gamma, const float* beta,
               const float* mean, const float* invstd, int training, int act, float* dy, float* dgamma,
               float* dbeta, long M, int C, float* ws, void* stream);
/* backward of y = dwconv(GLU(a)): da (B*T, 2C), dw (C,K) (=), db (C) (=). */
int cfm_glu_dwconv_bwd(const float* dy, const void* a, int dtype_a, const float* w_dw, void* da,
                       int dtype_da, float* dw, float* db, int B, int T, int C, int K, float* ws,
                       void* stream);
/* With dw == NULL, cfm_glu_dwconv_bwd leaves the depthwise weight/bias partial sums in ws; this
   reduces them (deterministically) into dw (C x K) and db (C) -- on any stream ordered after it. */
int cfm_glu_dwconv_bwd_wgrad(float* ws, int B, int T, int C, int K, float* dw, float* db, void* stream);
/* cfm_bn_silu_bwd_apply folded into cfm_glu_dwconv_bwd: the BatchNorm1d + SiLU input gradient
 *   dy = gamma*invstd*(du - dbeta*invM - yhat*dgamma*invM)   (training; eval: gamma*invstd*du)
 * is formed inside the depthwise backward from dz, y and the stats, never stored (torchaudio
 * ConformerLayer conv_module BatchNorm1d -> SiLU -> depthwise).  dbeta / dgamma:
 * from cfm_bn_silu_bwd_sums (or their SyncBatchNorm all-reduced totals with invM = 1 / rows summed
 * over).  K must be one of 3, 5, 7, 15, 31, 33.  dw == NULL: partials left in ws as above. */
int cfm_glu_dwconv_bwd_bn(const void* dz, int dtype_dz, const float* y, const float* gamma, const float* beta,
                          const float* mean, const float* invstd, const float* dbeta, const float* dgamma,
                          float invM, int training, const void* a, int dtype_a, const float* w_dw, void* da,
                          int dtype_da, float* dw, float* db, int B, int T, int C, int K, float* ws, void* stream);

/* ---------------------------------------------------------------- Attention
 * nn.MultiheadAttention(need_weights=False, key_padding_mask) core (torchaudio ConformerLayer
 * self_attn), optionally with Transformer-XL relative positions (transformers
 * Wav2Vec2ConformerSelfAttention, scores=((q+u)k^T + (q+v)p_{T-1-i+j}^T)/sqrt(dk)).
 * qkv: (B*T, 3*H*dk) rows [q | k | v]; o: (B*T, H*dk); lse: (B*H*T) fp32 log-sum-exp per query
 * (saved for backward); lengths: (B) int32 valid keys.  pos (rel only): (2T-1, H*dk) projected
 * table; pos_u / pos_v: (H*dk) fp32.  dtype: CFM_BF16 (MFMA) or CFM_F32. */
/* A/B switch (measurement only): bit 0 forces the tiled attention kernels instead of the
   whole-head ones (T <= 384: one workgroup per (b, h) with K/V staged once in LDS); bits 1-2 timing
   experiments of the whole-head forward (value 2: staging only, 4: no output stores -- outputs invalid);
   bit 4 runs bf16 relative-position attention on the SIMT kernels (parity cross-check); bit 6 keeps the
   rel-pos kernels' zero-filling (non-clamped) tile loads; bit 7 runs the round-4 rel-pos dpos kernel (one
   workgroup per (utterance, head, 64 relative rows); the round-5 kernel is checked against it). */
int cfm_attn_set_mode(int mode);
int cfm_attn_fwd(const void* qkv, void* o, float* lse, const int32_t* lengths, const void* pos,
                 const float* pos_u, const float* pos_v, int B, int T, int H, int dk, int dtype,
                 float drop_p, uint64_t seed, void* stream);
size_t cfm_attn_bwd_ws_bytes(int B, int T, int H, int dk, int rel, int dtype);
int cfm_attn_bwd(const void* qkv, const void* o, const void* dout, const float* lse,
                 const int32_t* lengths, const void* pos, const float* pos_u, const float* pos_v,
                 void* dqkv, float* dpos, float* dpos_u, float* dpos_v, int B, int T, int H,
                 int dk, int dtype, float drop_p, uint64_t seed, float* ws, void* stream);
/* The same with D = rowsum(dO * O) already in ws (cfm_gemm_desc.rowdot_* of the GEMM that produced dout):
   the D kernel is skipped.  bf16 MFMA path only (dk <= 64); rel-pos: ws is the full cfm_attn_bwd_ws_bytes
   workspace with D in its first B*H*T floats. */
int cfm_attn_bwd_with_d(const void* qkv, const void* o, const void* dout, const float* lse,
                        const int32_t* lengths, const void* pos, const float* pos_u, const float* pos_v,
                        void* dqkv, float* dpos, float* dpos_u, float* dpos_v, int B, int T, int H,
                        int dk, int dtype, float drop_p, uint64_t seed, float* ws, void* stream);
/* cfm_attn_bwd (d_ready 0) / cfm_attn_bwd_with_d (d_ready 1) with the projected-table gradient dpos written in
   dtype_dpos: CFM_F32, or CFM_BF16 on the rel-pos MFMA path (each fp32 column sum rounded as cfm_cast rounds
   it -- the compute-dtype copy the dW_pos GEMM reads, without an fp32 dpos and a cast pass).  d_ready bit 1 (round 6):
   ws is the full cfm_attn_bwd_ws_bytes workspace (D, if ready, in its first B*H*T floats) -- the non-rel whole-head
   path (T <= 384) then computes dQ from the dS^T its dK/dV kernel stores there (cfm_attn_bwd always does). */
int cfm_attn_bwd_ex(const void* qkv, const void* o, const void* dout, const float* lse,
                    const int32_t* lengths, const void* pos, const float* pos_u, const float* pos_v,
                    void* dqkv, void* dpos, int dtype_dpos, float* dpos_u, float* dpos_v, int B, int T,
                    int H, int dk, int dtype, float drop_p, uint64_t seed, int d_ready, float* ws,
                    void* stream);

/* ---------------------------------------------------------------- ConvSubSampling
 * lib/convsubsampling.py:16-45: Conv2d(1->C1, 7x7, s2) -> Conv2d(C1->C2, 3x3, s2), no padding.
 * conv1: x (B, F, T) fp32 -> h1 NHWC (B, F1, T1, C1) dtype_h; w1 (C1, 49), b1 (C1).
 * conv2: implicit GEMM over h1 -> h2 (B, T2, F2, C2) "frame-major" (row = (b,t2), features
 *        (f2, c2)) so the frame projection reads it as a plain (B*T2, F2*C2) matrix.
 *        w2r: (C2, 3*3*C1) reordered [c2][kh][kw][c1], dtype of h1. */
int cfm_conv1_fwd(const float* x, const float* w1, const float* b1, void* h1, int dtype_h, int B,
                  int F, int T, int C1, void* stream);
int cfm_conv2_fwd(const void* h1, const void* w2r, const float* b2, void* h2, int dtype_h2,
                  int dtype, int B, int F1, int T1, int C1, int C2, void* stream);
/* grads: dh1 from dh2 (transposed conv), dw2r (=), db2 via cfm_colsum; dw1 (=) and db1 (=). */
int cfm_conv2_bwd_data(const void* dh2, const void* w2r, void* dh1, int dtype, int B, int F1,
                       int T1, int C1, int C2, void* stream);
/* The same on the LDS-DMA GEMM pipeline: `ws` (cfm_conv2_bwd_data_ws_bytes) receives the per-parity-
   class K-major packing of w2r; NULL ws (or fp32) falls back to cfm_conv2_bwd_data. */
size_t cfm_conv2_bwd_data_ws_bytes(int C1, int C2);
int cfm_conv2_bwd_data_ws(const void* dh2, const void* w2r, void* dh1, int dtype, int B, int F1,
                          int T1, int C1, int C2, void* ws, void* stream);
int cfm_conv2_bwd_weight(const void* dh2, const void* h1, float* dw2r, int dtype, int B, int F1,
                         int T1, int C1, int C2, void* stream);
/* conv2 weight gradient with deterministic split-K slabs in `ws` (cfm_conv2_bwd_weight_ws_bytes bytes; NULL ->
 * one K slice): no atomics, no memset (graph-replay safe).  Replaces Conv2d.backward's weight gradient of
 * lib/convsubsampling.py:37. */
size_t cfm_conv2_bwd_weight_ws_bytes(int B, int F1, int T1, int C1, int C2);
int cfm_conv2_bwd_weight_ws(const void* dh2, const void* h1, float* dw2r, int dtype, int B, int F1,
                            int T1, int C1, int C2, float* ws, void* stream);
size_t cfm_conv1_bwd_ws_bytes(int B, int F, int T, int C1);
int cfm_conv1_bwd_weight(const void* dh1, int dtype_h, const float* x, float* dw1, float* db1,
                         int B, int F, int T, int C1, float* ws, void* stream);

/* ---------------------------------------------------------------- folded front-end ('frame' projection)
 * ConvSubSampling is two biased Conv2d with NO nonlinearity between them (lib/convsubsampling.py:41-43),
 * and in the 'frame' projection mode it feeds the per-frame Linear (the standard_linear of
 * asrnn.py:28,208 applied to every subsampled frame) before any dropout: the three are ONE linear map
 * of an Ke x Ke window of the mels, Ke = k1 + (k2 - 1) s1 (11), stride Se = s1 s2 (4):
 *   h[b, t2, o] = bfull[o] + sum_{f < Ke, r < F} Wfull[o][f][r] x[b, r, Se t2 + f]
 *   W_eff[c2][e][f] = sum_{c1, a, b} W2[c2][c1][a][b] W1[c1][e - s1 a][f - s1 b]       (the 11x11 conv)
 *   Wfull[o][f][r]  = sum_{f2, c2} Wp[o][f2 C2 + c2] W_eff[c2][r - Se f2][f]
 * so the step computes a (B*T2) x D x (Ke F) GEMM instead of conv1 -> conv2 -> Linear (~280 GFLOP
 * forward at Conformer-L / 15 s; the folded GEMM is 22 GFLOP with the hi + lo bf16 split of x).  The
 * GEMM reads x through a strided view: the packed input xt holds each utterance's frames as rows of Cx
 * channels (time-major; bf16 hi then lo rows of Fp, or fp32), row t2 of the view starts at frame Se t2
 * and spans Ke frames (lda = Se Cx < K: overlapping rows).  Utterance slots are Tslot = Se T2p frames
 * (T2p = T2 + padding rows), so the weight-gradient GEMM H = G^T X over all B*T2p padded rows (G zero
 * on the padding rows) is one single-stride product; the parameter gradients then follow from
 * H (D x Kp) and S = sum_rows G by the transposed contractions (cfm_ffold_bwd_weights).
 * Replaces Conv2d.forward/backward x2 and nn.Linear.forward/backward of that sequence. */
typedef struct {
  int B, F, T;        /* mels (B, F, T) fp32 */
  int C1, C2, D;      /* conv1 / conv2 channels, projection width */
  int k1, s1, k2, s2; /* square kernels, the same stride on both axes (nn.Conv2d, no padding) */
  int dtype;          /* GEMM operand type: CFM_BF16 or CFM_F32 */
  int hilo;           /* bf16: 1 = x as hi + lo bf16 rows (K doubles, ~16-bit x), 0 = hi only */
  /* filled by cfm_ffold_geometry: */
  int F2, T2, Ke, Se, Fp, Cx, Kp, lda, T2p, Tslot;
  long xt_elems;      /* elements of the packed input (B * Tslot * Cx + tail slack) */
  long ws_floats;     /* floats of the composed-weight workspace */
} cfm_ffold_geo;
int cfm_ffold_geometry(cfm_ffold_geo* g);
/* x (B, F, T) fp32 -> xt (xt_elems, dtype): frame t of utterance b at row b*Tslot + t (zero past T). */
int cfm_ffold_pack(const float* x, void* xt, const cfm_ffold_geo* g, void* stream);
/* w1 (C1, 1, k1, k1), b1 (C1), w2 (C2, C1, k2, k2), b2 (C2), wp (D, F2*C2) (features (f2, c2)), bp (D)
 * -> wfull (D, Kp) dtype (columns f*Cx + h*Fp + r, zero past Ke*Cx), bfull (D) fp32; ws (ws_floats) keeps
 * W_eff / b_eff for the backward. */
int cfm_ffold_compose(const float* w1, const float* b1, const float* w2, const float* b2, const float* wp,
                      const float* bp, void* wfull, float* bfull, float* ws, const cfm_ffold_geo* g,
                      void* stream);
/* H (D, Kp) fp32 = G^T X over the padded rows, S (D) = column sums of G (G: the gradient of h after the
 * dropout backward) -> dw1, db1, dw2, db2, dwp (same shapes as the weights; fp32, overwritten).  dbp = S. */
int cfm_ffold_bwd_weights(const float* H, const float* S, const float* w1, const float* b1, const float* w2,
                          const float* wp, float* ws, float* dw1, float* db1, float* dw2, float* db2, float* dwp,
                          const cfm_ffold_geo* g, void* stream);

/* ---------------------------------------------------------------- Adafactor (runner.py:36)
 * transformers.Adafactor(lr, beta1, scale_parameter=False, relative_step=False) as one
 * multi-tensor step.  The host fills a parameter table (cfm_adafactor_fill_table into a host
 * buffer of cfm_adafactor_table_bytes(n)), copies it to the device, and calls
 * cfm_adafactor_step with the prefix totals (factored rows, factored columns, elementwise
 * blocks = sum of cfm_adafactor_blocks(numel)).  col == NULL marks an unfactored (1-D) tensor,
 * whose full second moment lives in `row`.  rowmean: >= sum(nb) floats. */
size_t cfm_adafactor_table_bytes(int n_params);
int cfm_adafactor_fill_table(void* host_table, int i, float* p, const float* g, float* m, float* row,
                             float* col, long numel, int nb, int R, int C, long row_task_off,
                             long col_off, long blk_off, long rm_off, long rm_task_off,
                             long colpart_task_off, long part_off);
int cfm_adafactor_blocks(long numel);
long cfm_adafactor_row_tasks(int nb, int R, int C);
long cfm_adafactor_rowmean_tasks(int nb, int R);
long cfm_adafactor_colpart_tasks(int nb, int R, int C);
long cfm_adafactor_part_floats(int nb, int R, int C);
/* part: >= sum of cfm_adafactor_part_floats floats (column partials of wide matrices);
   partial: >= nblocks floats (per-block u^2 sums; RMS summed in block order, deterministic). */
int cfm_adafactor_step(const void* dev_table, int n, long nrow_tasks, long ncols, long nblocks,
                       long nrowmean_tasks, long ncolpart_tasks, float* rowmean, float* part,
                       float* partial, float lr, float beta1, float beta2t, float eps1, float clip,
                       void* stream);

/* ---------------------------------------------------------------- CTC head (runner.py:35,142-143)
 * Replaces torch.nn.CTCLoss(blank=hp.blank_idx, zero_infinity=True) on
 * log_softmax(final_fc(...)) (asrnn.py:45,256): log-softmax, alpha/beta recursions and the
 * gradient w.r.t. the logits, without host synchronisation (graph-capturable).
 * logits fp32, row (b, t) at logits + b*sb + t*st, classes contiguous (sb/st cover both the
 * reference's time-major (T, B, V) and batch-major layouts).  Feeding log-probabilities instead
 * of logits gives torch's result too (log_softmax is idempotent; the gradient is then exactly
 * torch's grad w.r.t. log_probs).  targets int32: utterance b at targets + tgt_off[b] (tgt_off
 * != NULL: torch's concatenated 1-D form) or targets + b*ldt (padded (B, ldt)); Smax >= every
 * target length.  in_len / tgt_len int32 on the device.
 * fwd: nll[b] = -log p(target_b | x_b), 0 where infinite and zero_infinity (torch semantics);
 *      ws: cfm_ctc_ws_bytes(B, T, Smax) bytes, read again by the backward.
 * bwd: grad[b, t, v] = (softmax - posterior) * grad_out[b * grad_out_stride] * r_b with
 *      r_b = 1 / (B * max(L_b, 1)) for reduction 1 (mean), 1 for 0 (none) / 2 (sum); zero for
 *      t >= in_len[b] and for zeroed infinite losses.  Output layout gsb/gst, dtype_grad f32|bf16. */
size_t cfm_ctc_ws_bytes(int B, int T, int Smax);
int cfm_ctc_loss_fwd(const float* logits, long sb, long st, const int32_t* targets, int ldt,
                     const int32_t* tgt_off, const int32_t* in_len, const int32_t* tgt_len, int B,
                     int T, int V, int Smax, int blank, int zero_infinity, float* nll, float* ws,
                     void* stream);
int cfm_ctc_loss_bwd(const float* logits, long sb, long st, const int32_t* targets, int ldt,
                     const int32_t* tgt_off, const int32_t* in_len, const int32_t* tgt_len, int B,
                     int T, int V, int Smax, int blank, int zero_infinity, const float* ws,
                     const float* grad_out, int grad_out_stride, int reduction, void* grad_logits,
                     int dtype_grad, long gsb, long gst, void* stream);

/* reduction='mean' of the forward's nll (torch.nn.CTCLoss: mean over b of nll[b] / max(tgt_len[b], 1)) as
 * ONE launch: *loss (fp32 scalar).  nonfinite (nullable): incremented by 1 when the mean is not finite (a
 * device step counter of bad steps, read once after a run).  Replaces the four element-wise passes of the
 * reduction and the host-side finiteness check's seven. */
int cfm_ctc_mean(const float* nll, const int32_t* tgt_len, int B, float* loss, int32_t* nonfinite,
                 void* stream);

/* Alpha / beta recursion health (no reference counterpart: the device recursion's own guard).  Each of the
 * recursion's inter-wave waits is bounded; a wait that gives up marks its direction aborted and the forward then
 * makes that utterance's nll NaN (so the loss and the logits gradient are NaN, never silently wrong).
 * cfm_ctc_bind_abort_counter(counter): int32 device counter (NULL unbinds) incremented once per aborted
 * utterance by every later cfm_ctc_loss_fwd -- told apart from genuine non-finite losses.
 * cfm_ctc_set_debug(mask): test hook, forces the abort path of the alpha (bit 0) / beta (bit 1) recursion. */
int cfm_ctc_bind_abort_counter(int32_t* counter);
int cfm_ctc_set_debug(int force_abort_mask);

/* Greedy decode: ASRNN.predict (asrnn.py:48-58, torch.argmax over classes: first maximum,
 * NaN wins) -> ids (B, T) int64; optionally (out, out_len != NULL) the Vocab.decode id filter
 * (myvocab.py:211-231): frames t < lens[b] (lens NULL: all T), ids equal to `blank` or `pad`
 * dropped (pad < 0: none), repeats collapsed first if `collapse` (the reference does not);
 * out (B, T) int32 padded with -1, out_len (B) int32. */
int cfm_ctc_greedy_decode(const float* logits, long sb, long st, const int32_t* lens, int B, int T,
                          int V, int blank, int pad, int collapse, int64_t* ids, int32_t* out,
                          int32_t* out_len, void* stream);

/* BiLSTM decoder recurrence: replaces the cuDNN/MIOpen recurrence of the
 * reference's nn.LSTM (asrnn.py:38 construct, :252 call on the 2-D encoder output = ONE unbatched
 * sequence of L = B*T_enc steps).  Gate order i, f, g, o (torch).  One cooperative launch per pass;
 * the input part x W_ih^T + b_ih + b_hh (gx) and the weight / input gradients are cfm_gemm calls.
 *   gx (L, ndir*4H) fp32, whh (ndir, 4H, H) fp32, y (L, ndir*H) = torch's output layout,
 *   gates (L, ndir*4H) post-activation, c (L, ndir*H) cell states (both saved for the backward),
 *   dg (L, ndir*4H) pre-activation gate gradients.  H % 8 == 0, H <= 1024, ndir 1 or 2.
 * ws: cfm_lstm_ws_bytes(H, ndir) of 16-B aligned device scratch (two error flags + the tagged-word
 * exchange rings; one workspace serves a forward and its backward): after a pass, ((int*)ws)[0] (fwd) /
 * ((int*)ws)[1] (bwd) != 0 means a step wait hit its 2-s limit. */
size_t cfm_lstm_ws_bytes(int H, int ndir);
int cfm_lstm_fwd(const float* gx, const float* whh, float* y, float* gates, float* c, int L, int H,
                 int ndir, void* ws, void* stream);
int cfm_lstm_bwd(const float* dy, const float* whh, const float* gates, const float* c, float* dg,
                 int L, int H, int ndir, void* ws, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CFM_H */
