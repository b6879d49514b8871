// logmel.hip — on-device log-mel front-end: waveform batch -> normalised log-mel
// batch in two launches, replacing the CPU librosa step of lib/standard/speechcommands.py:113-119:
//   mel = librosa.feature.melspectrogram(y, sr, n_mels)      periodic Hann, center=True (zero pad N/2),
//                                                             |rfft|^2, Slaney mel bank (norm='slaney')
//   mel = np.where(mel < 1e-10, 0, np.log(mel))              (:114)
//   mel -= min(mel); mel /= max(mel)                          (:117-119, per utterance)
// and the collate's zero padding of shorter utterances (speechcommands.py:188,198-210).
//
// logmel_frame_kernel: one workgroup per (frame, utterance).  The frame's N samples are read straight
// from the waveform (no framing copy: neighbouring frames overlap N/hop times and hit in L2), windowed
// and stored bit-reversed into LDS; an in-place radix-2 complex FFT (twiddles staged in LDS) gives the
// spectrum, |X_k|^2 lands in LDS, and each Slaney filter (a contiguous run of bins, tables built once on
// the host) is applied from there -> log -> one fp32 per (mel, frame), plus the frame's (min, max).
// logmel_norm_kernel: per utterance, reduce the frame partials, then (x - min) / (max - min) in place
// and zero the padded frames.  Both HBM-light (N/hop-fold L2 reuse of a few bytes per sample); the FFT
// is LDS/VALU work (5 N log2 N flops per frame).
#include "cfm_common.h"

namespace {

constexpr int LM_THREADS = 256;

__global__ __launch_bounds__(LM_THREADS) void logmel_frame_kernel(
    const float* __restrict__ wave, long ld_wave, const int32_t* __restrict__ lens, int logn, int hop,
    const float* __restrict__ window, const float2* __restrict__ twiddle, const int32_t* __restrict__ mel_lo,
    const int32_t* __restrict__ mel_cnt, const int32_t* __restrict__ mel_off, const float* __restrict__ mel_w,
    int n_mels, int nT, float* __restrict__ out, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char lm_lds[];
  const int N = 1 << logn, NB = N / 2 + 1;
  float2* buf = reinterpret_cast<float2*>(lm_lds);    // N complex
  float2* tw = buf + N;                                // N/2 twiddles exp(-2 pi i k / N)
  float* pw = reinterpret_cast<float*>(tw + N / 2);    // N/2 + 1 powers
  __shared__ float red[2][LM_THREADS / 64];
  const int t = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int len = lens[b];
  const int nTb = 1 + len / hop;                       // librosa: 1 + len // hop frames (center=True)
  float* ob = out + (long)b * n_mels * nT;
  if (t >= nTb) {                                      // padded frame (collate zeros)
    for (int m = tid; m < n_mels; m += LM_THREADS) ob[(long)m * nT + t] = 0.f;
    if (tid == 0) {
      part[((long)b * nT + t) * 2] = INFINITY;
      part[((long)b * nT + t) * 2 + 1] = -INFINITY;
    }
    return;
  }
  const float* wb = wave + (long)b * ld_wave;
  const long s0 = (long)t * hop - N / 2;               // center=True: N/2 zeros before sample 0
  for (int k = tid; k < N / 2; k += LM_THREADS) tw[k] = twiddle[k];
  for (int n = tid; n < N; n += LM_THREADS) {
    const long s = s0 + n;
    const float v = (s >= 0 && s < len) ? wb[s] * window[n] : 0.f;
    buf[__brev((unsigned)n) >> (32 - logn)] = make_float2(v, 0.f);
  }
  __syncthreads();
  // decimation-in-time butterflies, bit-reversed input -> natural-order output
  for (int lh = 0; lh < logn; ++lh) {
    const int half = 1 << lh;
    for (int j = tid; j < N / 2; j += LM_THREADS) {
      const int pos = j & (half - 1);
      const int i0 = ((j - pos) << 1) + pos, i1 = i0 + half;
      const float2 w = tw[pos << (logn - 1 - lh)];
      const float2 a = buf[i0], c = buf[i1];
      const float2 x = make_float2(w.x * c.x - w.y * c.y, w.x * c.y + w.y * c.x);
      buf[i0] = make_float2(a.x + x.x, a.y + x.y);
      buf[i1] = make_float2(a.x - x.x, a.y - x.y);
    }
    __syncthreads();
  }
  for (int k = tid; k < NB; k += LM_THREADS) {
    const float2 x = buf[k];
    pw[k] = x.x * x.x + x.y * x.y;
  }
  __syncthreads();
  float mn = INFINITY, mx = -INFINITY;
  for (int m = tid; m < n_mels; m += LM_THREADS) {
    const int lo = mel_lo[m], cnt = mel_cnt[m], off = mel_off[m];
    float acc = 0.f;
    for (int i = 0; i < cnt; ++i) acc = fmaf(mel_w[off + i], pw[lo + i], acc);
    const float v = acc < 1e-10f ? 0.f : logf(acc);
    ob[(long)m * nT + t] = v;
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  mx = wave_max(mx);
  mn = -wave_max(-mn);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = mn;
    red[1][tid >> 6] = mx;
  }
  __syncthreads();
  if (tid == 0) {
    float a = red[0][0], c = red[1][0];
    for (int w = 1; w < LM_THREADS / 64; ++w) {
      a = fminf(a, red[0][w]);
      c = fmaxf(c, red[1][w]);
    }
    part[((long)b * nT + t) * 2] = a;
    part[((long)b * nT + t) * 2 + 1] = c;
  }
}

// grid (chunks, B): every workgroup reduces its utterance's frame partials (nT pairs, L2-resident), then
// normalises its slice of the utterance's (n_mels x nT) block; padded frames stay 0
__global__ __launch_bounds__(LM_THREADS) void logmel_norm_kernel(float* __restrict__ out, const float* __restrict__ part,
                                                                 const int32_t* __restrict__ lens, int hop, int n_mels,
                                                                 int nT) {
  __shared__ float red[2][LM_THREADS / 64];
  const int b = blockIdx.y, tid = threadIdx.x;
  const int nTb = min(nT, 1 + lens[b] / hop);
  float mn = INFINITY, mx = -INFINITY;
  for (int t = tid; t < nTb; t += LM_THREADS) {
    mn = fminf(mn, part[((long)b * nT + t) * 2]);
    mx = fmaxf(mx, part[((long)b * nT + t) * 2 + 1]);
  }
  mx = wave_max(mx);
  mn = -wave_max(-mn);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = mn;
    red[1][tid >> 6] = mx;
  }
  __syncthreads();
  mn = red[0][0];
  mx = red[1][0];
  for (int w = 1; w < LM_THREADS / 64; ++w) {
    mn = fminf(mn, red[0][w]);
    mx = fmaxf(mx, red[1][w]);
  }
  const float span = mx - mn;                          // == max(x - mn) in fp32 (rounding is monotone)
  float* ob = out + (long)b * n_mels * nT;
  const long total = (long)n_mels * nT;
  for (long i = (long)blockIdx.x * LM_THREADS + tid; i < total; i += (long)gridDim.x * LM_THREADS) {
    const int t = (int)(i % nT);
    if (t < nTb) ob[i] = (ob[i] - mn) / span;
  }
}

}  // namespace

CFM_EXPORT size_t cfm_logmel_ws_bytes(int B, int nT) { return (size_t)B * (size_t)nT * 2 * sizeof(float); }

CFM_EXPORT int cfm_logmel_fwd(const float* wave, long ld_wave, const int32_t* lens, int B, int n_fft, int hop,
                              const float* window, const float* twiddle, const int32_t* mel_lo, const int32_t* mel_cnt,
                              const int32_t* mel_off, const float* mel_w, int n_mels, int nT, int normalize, float* out,
                              float* ws, void* stream) {
  CFM_REQUIRE(wave && lens && window && twiddle && mel_lo && mel_cnt && mel_off && mel_w && out && ws, CFM_ERR_ARG,
              "null pointer");
  CFM_REQUIRE(n_fft >= 16 && n_fft <= 4096 && (n_fft & (n_fft - 1)) == 0, CFM_ERR_SHAPE,
              "n_fft must be a power of two in [16, 4096]");
  CFM_REQUIRE(B >= 0 && hop > 0 && n_mels > 0 && nT >= 0 && ld_wave >= 0, CFM_ERR_SHAPE, "bad shape");
  CFM_REQUIRE(nT <= 65535 && B <= 65535, CFM_ERR_SHAPE, "grid too large");
  if (B == 0 || nT == 0) return CFM_OK;
  int logn = 0;
  while ((1 << logn) < n_fft) ++logn;
  const size_t lds = (size_t)n_fft * 8 + (size_t)(n_fft / 2) * 8 + (size_t)(n_fft / 2 + 1) * 4;
  hipStream_t s = cfm::as_stream(stream);
  hipLaunchKernelGGL(logmel_frame_kernel, dim3((unsigned)nT, (unsigned)B), dim3(LM_THREADS), lds, s, wave, ld_wave,
                     lens, logn, hop, window, reinterpret_cast<const float2*>(twiddle), mel_lo, mel_cnt, mel_off,
                     mel_w, n_mels, nT, out, ws);
  if (normalize) {
    const long total = (long)n_mels * nT;
    int chunks = (int)((total + LM_THREADS * 8 - 1) / (LM_THREADS * 8));
    if (chunks > 256) chunks = 256;
    if (chunks < 1) chunks = 1;
    hipLaunchKernelGGL(logmel_norm_kernel, dim3((unsigned)chunks, (unsigned)B), dim3(LM_THREADS), 0, s, out, ws,
                       lens, hop, n_mels, nT);
  }
  return cfm::check_launch("cfm_logmel_fwd");
}
