/*
 * lq_kernels.h -- the thin C-ABI between the C host objects (host/ *.c) and the
 * hand-written HIP kernels (csrc/ *.hip).  Plain pointers and sizes only.
 *
 * Device pointers are `void *` (complex samples are interleaved float pairs,
 * 8 bytes).  Every launcher enqueues on the given HIP stream and returns
 * immediately; errors abort with a message (lqrt_check).
 */
#ifndef LQ_KERNELS_H
#define LQ_KERNELS_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- runtime */
void   lqrt_require_device(const char *who);    /* abort if no usable GPU */
void  *lqrt_malloc(size_t bytes);               /* device memory, zeroed   */
void   lqrt_free(void *p);
void  *lqrt_host_alloc(size_t bytes);           /* pinned host memory      */
void   lqrt_host_free(void *p);
void  *lqrt_stream_create(void);
void   lqrt_stream_destroy(void *s);
void   lqrt_h2d(void *dst, const void *src, size_t bytes, void *stream);
void   lqrt_d2h(void *dst, const void *src, size_t bytes, void *stream);
void   lqrt_d2d(void *dst, const void *src, size_t bytes, void *stream);
void   lqrt_memset(void *dst, size_t bytes, void *stream);
void   lqrt_sync(void *stream);
void   lqrt_device_sync(void);
int    lqrt_is_device_ptr(const void *p);
const float *lqrt_twiddles(void);               /* W_4096^e = exp(-2 pi i e/4096), e<4096 */
#define LQRT_ZEROS 256
const float *lqrt_zeros(void);                  /* LQRT_ZEROS bytes of zeros in device memory */
/* small-call completion: one kernel copies `bytes` (a multiple of 4, at most
 * LQRT_COPYOUT_MAX) from device memory src to pinned host memory dst, makes
 * them visible system-wide and then stores `seq` to the pinned word *flag;
 * lqrt_wait_flag spins until it sees seq (then falls back to a stream sync,
 * which also reports a kernel fault). */
#define LQRT_COPYOUT_MAX (64u << 10)
void   lqrt_copyout_signal(const void *src, void *dst, size_t bytes, unsigned *flag, unsigned seq, void *stream);
void   lqrt_wait_flag(const unsigned *flag, unsigned seq, void *stream);

/* ---------------------------------------------------------------- dotprod
 * Y[v] = sum_i h[i] X[v*stride + i], v < nvec.  kind: 0 rrrf, 1 crcf, 2 cccf */
void lqk_dotprod_batch(int kind, const void *h, unsigned int n, const void *X,
                       unsigned long long stride, unsigned long long nvec, void *Y, void *stream);
/* one dot product (dotprod_*_execute): x may be pinned host memory, y is
 * pinned host memory, *flag = seq is raised once y is visible to the host */
void lqk_dotprod_single(int kind, const void *h, unsigned int n, const void *x, void *y, unsigned *flag,
                        unsigned seq, void *stream);

/* ---------------------------------------------------------------- firfilt
 * Streaming FIR: y[i] = scale * sum_{k<hlen} h[k] ext[i-k], where ext[t] = x[t]
 * for t >= 0 and win[HP+t] for t < 0 (win = the previous HP = hc*nchunk
 * inputs, oldest first, 16-byte aligned).  hpad: coefficients in natural order, zero padded to
 * nchunk*hc.  kind: 0 rrrf, 1 crcf, 2 cccf.  x == y allowed (in-place). */
typedef struct {
    int kind;
    unsigned int hlen;       /* logical length */
    unsigned int hc;         /* compile-time chunk class: 8,16,32,64 */
    unsigned int nchunk;     /* padded length = hc*nchunk */
    const void *hpad;        /* device coefficients (float or float2) */
    float scale_re, scale_im;
    int mx_ok;               /* taps finite, nonzero |h| in [2^-50, 2^50]: the matrix-core kernel's
                              * three-term bf16 split is float32-accurate (k_firfilt_mx.hip) */
} lqk_fir_desc;

/* A stream object's history update folded into its stream kernel: dst =
 * the last L samples of (src: L samples) ++ (x: n samples), what
 * lqk_window_append does as a launch of its own (~5 us per call, measured in
 * the round-6 rocprof trace).  The kernel's workgroups copy grid-strided
 * slices of it before their own work; dst == NULL: no job. */
typedef struct {
    const void *src;
    const void *x;
    unsigned long long n;
    void *dst;
    unsigned int L;
} lqk_hist_job;

/* job (NULL: none): the window update, done inside the matrix-core kernel
 * when it takes the call, else launched before the VALU kernel (which may
 * run in place) */
void lqk_firfilt(const lqk_fir_desc *d, const void *hist, const void *x, unsigned long long n,
                 void *y, void *scratch, const lqk_hist_job *job, void *stream);
/* crcf with 33..64 taps on the matrix cores (k_firfilt_mx.hip); returns 0
 * when the call does not qualify (then lqk_firfilt runs the VALU kernel) */
int lqk_firfilt_mx(const lqk_fir_desc *d, const void *hist, const void *x, unsigned long long n, void *y,
                   const lqk_hist_job *job, void *stream);
/* bytes of scratch lqk_firfilt needs for an in-place call of n samples */
size_t lqk_firfilt_scratch_bytes(const lqk_fir_desc *d, unsigned long long n);
/* longest history (padded tap count) the direct FIR kernel can hold in LDS */
unsigned int lqk_firfilt_max_history(int kind);

/* window maintenance: dst[0..L) = last L samples of (src_hist[0..L) ++ x[0..n)) */
void lqk_window_append(int is_complex, const void *src_hist, unsigned int L, const void *x,
                       unsigned long long n, void *dst_hist, void *stream);

/* one output of a dot product of hr (reversed coefficients, hlen) against
 * win (oldest first), times scale: the per-sample firfilt_execute() path.
 * With a flag, y is pinned host memory and the kernel raises *flag = seq
 * once y is visible to the host (see lqrt_wait_flag); flag may be NULL. */
void lqk_fir_single(const lqk_fir_desc *d, const void *win, void *y, unsigned *flag, unsigned seq, void *stream);

/* ---------------------------------------------------------------- firdecim / firinterp
 * decim: y[o] = sum_k h[k] ext[o*M + phase - k]  (o < nout)
 * interp: y[i*M + p] = scale * sum_{l<L} h[p + l*M] ext[i - l]  (i < n) */
void lqk_firdecim(const lqk_fir_desc *d, unsigned int M, const void *hist, const void *x,
                  unsigned long long nout, void *y, void *stream);
/* phase-layout decimator: hq = M x QC phase-major padded taps,
 * hq[r*QC + q] = h[q*M + r] (0 past hlen), QC = lqk_firdecim_ph_qc(M, hlen);
 * hist = the previous hl1 = hlen-1 inputs.  Returns -1 (nothing launched)
 * when the tile does not fit in LDS. */
unsigned lqk_firdecim_ph_qc(unsigned M, unsigned hlen);
int lqk_firdecim_ph(int kind, unsigned int M, unsigned int QC, const void *hq, unsigned int hl1,
                    const void *hist, const void *x, unsigned long long nout, void *y, void *stream);
void lqk_firinterp(int kind, const void *hpoly /* M x L, h[p + l*M] */, unsigned int M,
                   unsigned int L, float scale_re, float scale_im, const void *hist, const void *x,
                   unsigned long long n, void *y, void *stream);

/* ---------------------------------------------------------------- firpfbch2 analyzer
 * nblocks consecutive analyzer blocks over x (nblocks*M/2 samples); hist holds
 * the previous 2*m*M - M/2 inputs; p0 = parity of the first block.
 * hsub: M x 2m table, hsub[i*2m + n] = h[i + n*M].  Y: nblocks x M, already
 * divided by M (firpfbch2.c:277-278). */
void lqk_firpfbch2_analyzer(unsigned int M, unsigned int m, const void *hsub, const void *hist,
                            const void *x, unsigned long long nblocks, int p0, void *Y,
                            void *stream);
/* M = 1024 (m = 2 or 4) register/LDS-streaming fast path; returns 0 if the
 * shape is not covered (caller then uses lqk_firpfbch2_analyzer).  B0 = global
 * index of the first block (only its parity matters).  hsub here is the tap
 * table already multiplied by 1/M (the kernel applies no output scale). */
/* firpfbch_crcf analyzer M = 1024, p in {4, 8}, real taps (k_pfb2_fast.hip); 0 = not handled */
int lqk_firpfbch_analyzer_fast(int ctaps, unsigned int M, unsigned int p, const void *hsub, const void *hist,
                               const void *x, unsigned long long nblocks, void *Y, void *stream);
/* firpfbch_crcf synthesizer M = 1024, p in {4, 8}, real taps, nblocks >= p-1; 0 = not handled */
int lqk_firpfbch_synthesizer_fast(int ctaps, unsigned int M, unsigned int p, const void *hsub, void *state,
                                  const void *X, unsigned long long nblocks, void *y, void *stream);
/* firpfbch2_crcf synthesizer M = 1024, m in {2, 4}, nblocks >= 4m-1; 0 = not handled */
int lqk_firpfbch2_synthesizer_fast(unsigned int M, unsigned int m, const void *hsub, void *state, const void *X,
                                   unsigned long long nblocks, int p0, void *Y, void *stream);
/* batched transforms with the two sequential output scales of fft_batch_scaled (k_channelizer.hip) */
void lqk_fft_batch_scaled(unsigned int n, int dir, const void *x, void *y, unsigned long long batch, float s1,
                          float s2, void *stream);
/* job (NULL: none) is done only when the call is handled (returns 1).
 * flag (NULL: none): Y is pinned host memory, and the kernel raises *flag =
 * seq (system scope) once Y is visible to the host -- for calls that take a
 * single workgroup (a few blocks), else 0 is returned before any launch */
int lqk_firpfbch2_analyzer_fast(unsigned int M, unsigned int m, const void *hsub, const void *hist,
                                const void *x, unsigned long long nblocks, long long B0, void *Y,
                                const lqk_hist_job *job, unsigned *flag, unsigned seq, void *stream);
/* synthesizer: nblocks x M channel inputs -> nblocks x M/2 outputs.
 * state: the previous 4m-1 IFFT vectors (M each), zscratch (4m-1+nblocks)*M;
 * see csrc/k_channelizer.hip */
void lqk_firpfbch2_synthesizer(unsigned int M, unsigned int m, const void *hsub_syn,
                               void *state, void *zscratch, const void *X,
                               unsigned long long nblocks, int p0, void *Y, void *stream);

/* ---------------------------------------------------------------- firpfbch (critically sampled)
 * analyzer: block b consumes x[bM .. bM+M); window i receives x[bM + M-1-i]
 * X[M-1-i] = sum_n h[i + n*M] win_i, Y = FFT_forward(X).  hsub[i*p + n] = h[i+n*M];
 * ctaps: hsub holds complex taps (cccf), else real (crcf) */
/* firpfbch analyzer M = 1024 (crcf, p in {4, 8}), calls of <= 16 blocks in
 * one workgroup, with the history job and, optionally, the completion flag
 * (Y pinned host memory; see lqk_firpfbch2_analyzer_fast); 0: not handled */
int lqk_firpfbch_analyzer_few(int ctaps, unsigned int M, unsigned int p, const void *hsub, const void *hist,
                              const void *x, unsigned long long nblocks, void *Y, const lqk_hist_job *job,
                              unsigned *flag, unsigned seq, void *stream);
void lqk_firpfbch_analyzer(int ctaps, unsigned int M, unsigned int p, const void *hsub, const void *hist,
                           const void *x, unsigned long long nblocks, void *Y, void *stream);
void lqk_firpfbch_synthesizer(int ctaps, unsigned int M, unsigned int p, const void *hsub, void *state,
                              void *zscratch, const void *X, unsigned long long nblocks, void *y,
                              void *stream);

/* ---------------------------------------------------------------- FFT / fftfilt */
/* batched complex FFT of power-of-two size n (2..4096): dir +1 forward, -1 backward */
void lqk_fft_batch(unsigned int n, int dir, const void *x, void *y, unsigned long long batch,
                   void *stream);
/* overlap-save fast convolution: y[t] = scale * sum_k h[k] ext[t-k], t < n;
 * nfft = lqk_fftfilt_nfft(real_io, hlen) (4096-point segments up to 2049
 * taps, 8192 for complex I/O up to 4097 taps, 0: too long);
 * H = FFT_nfft(h zero padded) (unscaled, lqk_fftfilt_make_H); scale = the
 * user scale; hist = previous hlen-1 inputs.  x must not alias y.
 * guard (complex I/O only): 0 fftfilt; 1 / 2 firfilt crcf / cccf --
 * segments whose inputs hold Inf / NaN, |v| > 2^100 or nonzero |v| < 2^-60
 * are recomputed as the direct convolution over hx (the natural-order taps,
 * hlen); flags: device scratch of lqk_fftfilt_flag_bytes(). */
unsigned int lqk_fftfilt_nfft(int real_io, unsigned int hlen);
size_t lqk_fftfilt_flag_bytes(unsigned int hlen, unsigned int nfft, unsigned long long n);
void lqk_fftfilt_run(int real_io, unsigned int hlen, unsigned int nfft, const void *H, const void *hist,
                     const void *x, unsigned long long n, void *y, float scale_re, float scale_im,
                     const float *hx, int guard, void *flags, const lqk_hist_job *job, void *stream);
void lqk_fftfilt_make_H(const void *h_dev, unsigned int hlen, int is_complex, unsigned int nfft, void *H,
                        void *stream);

/* ---------------------------------------------------------------- resamp / firpfb
 * Timing plan: checkpoint c = the resampler's timing state before plan input
 * c*LQK_RS_CK and K = outputs emitted by the plan's inputs before it; the
 * state at any other input is the checkpoint before it stepped forward
 * (< LQK_RS_CK inputs).  Power-of-two bank counts store (tau, K) -- the rest
 * of the state is a function of tau there (host/resamp.c) -- other bank
 * counts the whole state (tau, mu, b, state; bst = b*2 + (state == INTERP)).
 * Inputs g >= pre repeat with period P (Q outputs per period): state(g) =
 * state(pre + (g-pre) % P), K += Q per period; positions beyond `end` are
 * clamped to it (direct plans cover end + 1 positions). */
#define LQK_RS_CK 4   /* a checkpoint per replay lane's 4 inputs (csrc/k_resamp.hip k_resamp3) */
typedef struct {
    float tau, mu;
    int bst;
    unsigned int K;
} lqk_rs_entry;
typedef struct {
    float tau;
    unsigned int K;
} lqk_rs_entry_p2;
typedef struct {
    const void *tab;           /* device: lqk_rs_entry_p2[] (p2) or lqk_rs_entry[], checkpoint c at [c] */
    unsigned long long pre, P, Q;
    unsigned long long end;
    int p2;
} lqk_rs_plan;
/* n inputs x (plan positions g0 .. g0+n) -> the nout outputs y[K(g) - K0 ...]
 * (n <= LQK_RS_MAXN, nout * sample size < 2^31);
 * taps: npfb x L pairs (h[b + n*npfb], h[(b+1)%npfb + n*npfb]); hist = last L inputs.
 * real_io: float samples (rrrf), else interleaved complex (crcf, cccf: the taps are real for every type) */
#define LQK_RS_MAXN (1ull << 27)
void lqk_resamp(int real_io, const lqk_rs_plan *pl, unsigned long long g0, unsigned long long K0, unsigned int npfb,
                unsigned int L, float del, const void *taps, const void *taps2, const void *hist, const void *x,
                unsigned long long n, void *y, unsigned long long nout, void *stream);
/* taps2: (npfb+1) x LP pairs, LP = (L+3) & ~1: row b < npfb (h_b[L-p], h_{b+1}[L-p]) for p = 1..L, row
 * npfb the BOUNDARY pair (h_{npfb-1}[L-1-p], h_0[L-p]); zero elsewhere (NULL: untiled kernel) */
/* Output plan of k_resamp4 (csrc/k_resamp4.hip: complex samples, power-of-two
 * npfb, 1/4 < r <= npfb with one or two outputs per input (any number past
 * r = 2), or an output every one or two (two to four below r = 1/2) inputs,
 * over the whole plan):
 * entries {tau, i} = the timing phase at which a plan output is emitted and
 * the plan input it belongs to -- tab[c] for output 4c (c < npre =
 * ceil(pre / 4)), then tab[npre + c] for output pre + 4c within one period.
 * Outputs k >= pre repeat with period QT outputs / PT inputs (QT >= 256):
 * state(k) = state(pre + (k - pre) % QT) with i += PT per period; pre = ~0:
 * no period (a direct plan; ntab entries cover the plan's outputs). */
typedef struct {
    float tau;
    unsigned int i;
} lqk_rs4_entry;
typedef struct {
    const void *tab;              /* device lqk_rs4_entry[ntab] */
    unsigned long long ntab;
    unsigned long long pre, npre, QT, PT;
} lqk_rs4_plan;
/* msresamp's interpolating chain fused into k_resamp4: the resampler's
 * outputs u feed one half-band interpolator stage (resamp2 interp mode,
 * src/filter/src/resamp2.c:330-360) in registers -- y[2k] = u[k - m],
 * y[2k+1] = sum_j h1[j] u[k+1+j-2m] -- and never reach HBM.  hist: the
 * stage's window before the call (2m samples, oldest first, both of its
 * windows hold the same pushes in interp mode); hist_new0 / hist_new1: its two
 * windows after the call (written by the kernel; nout >= 1). */
#define LQK_RS4_HB_MAXM 12
typedef struct {
    int m;                        /* semi-length: 3 .. LQK_RS4_HB_MAXM */
    float h1[2 * LQK_RS4_HB_MAXM];/* odd taps h1[j] = h[4m-1-2j] (real) */
    const void *hist;
    void *hist_new0, *hist_new1;
} lqk_rs4_hb;
int lqk_resamp4_supported(unsigned int npfb, unsigned int L);
/* the fused chain's shapes: L = 14, npfb = 64, 1 < r < 2, m in 3 .. LQK_RS4_HB_MAXM */
int lqk_resamp4_hb_supported(unsigned int npfb, unsigned int L, float del, int m);
/* n complex inputs x (plan inputs g0 .. g0+n) -> the nout outputs y[k - K0]
 * for plan outputs k = K0 .. K0+nout-1; taps2 and hist as lqk_resamp.  hb
 * (NULL: none): y receives the half-band stage's 2 nout outputs instead */
void lqk_resamp4(const lqk_rs4_plan *pl, unsigned long long g0, unsigned long long K0, unsigned int npfb,
                 unsigned int L, float del, const void *taps2, const void *hist, const void *x, unsigned long long n,
                 void *y, unsigned long long nout, const lqk_rs4_hb *hb, const lqk_hist_job *job, void *stream);
/* firpfb_execute(i): y = scale * sum_n hpoly[i*L + n] win[L-1-n] (win: L samples, oldest first) */
void lqk_firpfb_single(int kind, const void *hpoly, unsigned int L, unsigned int i, const void *win,
                       float scale_re, float scale_im, void *y, unsigned *flag, unsigned seq, void *stream);

/* ---------------------------------------------------------------- FFT of any size (csrc/k_fft.hip)
 * batch transforms of n points (complex, contiguous), dir +1 forward / -1
 * backward, unnormalised; x may alias y.  work: lqk_fft_work_bytes(n, batch)
 * bytes of device scratch (NULL when 0). */
size_t lqk_fft_work_bytes(unsigned int n, unsigned long long batch);
void lqk_fft_any(unsigned int n, int dir, const void *x, void *y, unsigned long long batch, void *work,
                 void *stream);
/* real-to-real (fft_r2r_1d.c): type codes as liquid_fft_type (10-13 DCT, 20-23 DST); x must not alias y */
enum {
    LQK_R2R_REDFT00 = 10, LQK_R2R_REDFT10 = 11, LQK_R2R_REDFT01 = 12, LQK_R2R_REDFT11 = 13,
    LQK_R2R_RODFT00 = 20, LQK_R2R_RODFT10 = 21, LQK_R2R_RODFT01 = 22, LQK_R2R_RODFT11 = 23,
};
void lqk_fft_r2r(int type, unsigned int n, const void *x, void *y, unsigned long long batch, void *stream);

/* ---------------------------------------------------------------- spgram (csrc/k_spgram.hip)
 * gather: out[t][i] = ext[ends[t]+1+i] w[i] (i < W, zero to nfft), ext = hist(W) ++ x;
 * accumulate: psd = (1-a) psd + a |X_t|^2 in t order; sum: acc[shift(k)] += sum_t |X_t[k]|^2;
 * db: mode 0 10log10(|X|^2+1e-16) shifted, 1 10log10(v) shifted, 2 10log10(v/T) */
void lqk_spgram_gather(int real_in, const void *hist, unsigned int W, const void *x, const long long *ends,
                       unsigned long long T, const float *w, unsigned int nfft, void *out, void *stream);
/* per-bin reductions over T transforms; work: lqk_spgram_work_bytes(T, nfft) bytes of device scratch */
size_t lqk_spgram_work_bytes(unsigned long long T, unsigned int nfft);
void lqk_spgram_accumulate(const void *X, unsigned long long T, unsigned int nfft, float alpha, float *psd,
                           void *work, void *stream);
void lqk_spgram_sum(const void *X, unsigned long long T, unsigned int nfft, float *acc, void *work, void *stream);
/* nfft = 1024 (W <= 1024): windows gathered from (hist | x), transformed and reduced in one pass;
 * transform t ends at e0 + t*hop (the last at elast); accum: dst = psd (exponential average),
 * else dst = acc (sum, fft-shifted); work: lqk_spgram_work_bytes(T, 1024) bytes */
void lqk_spgram_fused1024(int real_in, const void *hist, unsigned int W, const void *x, long long e0,
                          long long hop, unsigned long long T, long long elast, const float *w, int accum,
                          float alpha, float *dst, void *work, void *stream);
void lqk_spgram_db(int mode, const void *X, const float *v, unsigned int nfft, float T, float *out, void *stream);

/* ---------------------------------------------------------------- resamp2 (half-band)
 * n calls of one resamp2 mode (src/filter/src/resamp2.c:273-356).  hist0/hist1 =
 * the two 2m-sample windows (oldest first); the updated windows go to
 * hist0_new/hist1_new (must not alias).  taps: the 2m odd taps h1[j] = h[4m-1-2j]
 * (float for kind 0/1, float2 for kind 2).  Outputs: filter y0[i], y1[i];
 * decim y0[i] (times scale, a power of two); analyzer/interp/synthesizer
 * y0[2i], y0[2i+1].  t0: filter-mode toggle before the first call. */
enum { LQK_R2_FILTER = 0, LQK_R2_ANALYZER, LQK_R2_SYNTHESIZER, LQK_R2_DECIM, LQK_R2_INTERP };
void lqk_resamp2(int kind, int mode, unsigned int m, int t0, float scale, const void *taps, const void *hist0,
                 const void *hist1, void *hist0_new, void *hist1_new, const void *x, unsigned long long n,
                 void *y0, void *y1, void *stream);

#ifdef __cplusplus
}
#endif

#endif
