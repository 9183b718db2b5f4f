/*
 * liquid_mi355x.h -- drop-in replacement for the streaming filter /
 * channelizer subset of liquid-dsp's include/liquid.h (liquid-dsp 1.2.0),
 * executed on AMD Instinct MI355X (gfx950) by hand-written HIP kernels.
 *
 * Every declaration in the "liquid.h subset" sections keeps the reference
 * signature and semantics (create / execute / destroy, opaque handles,
 * unsigned sizes, liquid_float_complex samples, invalid arguments print to
 * stderr and exit(1)).  The line references name the liquid.h declaration
 * each symbol replaces.  A program that only uses these objects compiles
 * against this header unchanged and links -lliquid_mi355x instead of
 * -lliquid.
 *
 * The "extensions" sections are additive (new names): batched and
 * device-pointer entry points, explicit stream control.  liquid.h's per-call
 * granularity (e.g. firpfbch2_crcf_execute = M/2 samples) cannot feed a GPU;
 * the block/batch forms can.  All original symbols still return only after
 * their output is written.
 *
 * There is no CPU fallback: without a usable HIP device every constructor
 * prints an error and exits (same failure style as the reference).
 */
#ifndef LIQUID_MI355X_H
#define LIQUID_MI355X_H

#ifdef __cplusplus
extern "C" {
#define LIQUID_USE_COMPLEX_H 0
#else
#define LIQUID_USE_COMPLEX_H 1
#endif

/* liquid.h:49-50 */
#define LIQUID_VERSION "1.2.0"
#define LIQUID_VERSION_NUMBER 1002000

/* liquid.h:55-57 */
extern const char liquid_version[];
const char *liquid_libversion(void);
int liquid_libversion_number(void);

/* liquid.h:77-88: C99 complex in C, std::complex<float> in C++ (same layout) */
#if LIQUID_USE_COMPLEX_H == 1
#include <complex.h>
#define LIQUID_DEFINE_COMPLEX(R, C) typedef R _Complex C
#elif defined _GLIBCXX_COMPLEX || defined _LIBCPP_COMPLEX
#define LIQUID_DEFINE_COMPLEX(R, C) typedef std::complex<R> C
#else
#define LIQUID_DEFINE_COMPLEX(R, C) typedef struct { R real; R imag; } C;
#endif
LIQUID_DEFINE_COMPLEX(float, liquid_float_complex);

/* liquid.h:6662 (src/utility/src/msb_index.c:110-135): index of the most
   significant set bit, 1-based (floor(log2 x)+1), 0 for x = 0 */
unsigned int liquid_msb_index(unsigned int _x);

/* liquid.h:5651-5652 */
#define LIQUID_ANALYZER 0
#define LIQUID_SYNTHESIZER 1

/* ------------------------------------------------------------------------ */
/* filter design (liquid.h:1476 kaiser_beta_As, :1548 liquid_firdes_kaiser)  */
/* ------------------------------------------------------------------------ */
float kaiser_beta_As(float _As);
void liquid_firdes_kaiser(unsigned int _n, float _fc, float _As, float _mu, float *_h);
/* liquid.h:1413-1435: prototype filter types */
typedef enum {
    LIQUID_FIRFILT_UNKNOWN = 0,
    LIQUID_FIRFILT_KAISER,
    LIQUID_FIRFILT_PM,
    LIQUID_FIRFILT_RCOS,
    LIQUID_FIRFILT_FEXP,
    LIQUID_FIRFILT_FSECH,
    LIQUID_FIRFILT_FARCSECH,
    LIQUID_FIRFILT_ARKAISER,
    LIQUID_FIRFILT_RKAISER,
    LIQUID_FIRFILT_RRC,
    LIQUID_FIRFILT_hM3,
    LIQUID_FIRFILT_GMSKTX,
    LIQUID_FIRFILT_GMSKRX,
    LIQUID_FIRFILT_RFEXP,
    LIQUID_FIRFILT_RFSECH,
    LIQUID_FIRFILT_RFARCSECH,
} liquid_firfilt_type;
/* liquid.h:1444-1471 */
void liquid_firdes_prototype(liquid_firfilt_type _type, unsigned int _k, unsigned int _m, float _beta, float _dt,
                             float *_h);
int liquid_getopt_str2firfilt(const char *_str);
unsigned int estimate_req_filter_len(float _df, float _As);
float estimate_req_filter_As(float _df, unsigned int _N);
float estimate_req_filter_df(float _As, unsigned int _N);
/* liquid.h:1481-1512: Parks-McClellan (this build designs band-pass filters) */
typedef enum {
    LIQUID_FIRDESPM_BANDPASS = 0,
    LIQUID_FIRDESPM_DIFFERENTIATOR,
    LIQUID_FIRDESPM_HILBERT
} liquid_firdespm_btype;
typedef enum {
    LIQUID_FIRDESPM_FLATWEIGHT = 0,
    LIQUID_FIRDESPM_EXPWEIGHT,
    LIQUID_FIRDESPM_LINWEIGHT,
} liquid_firdespm_wtype;
void firdespm_run(unsigned int _h_len, unsigned int _num_bands, float *_bands, float *_des, float *_weights,
                  liquid_firdespm_wtype *_wtype, liquid_firdespm_btype _btype, float *_h);
/* liquid.h:1573-1605 */
void liquid_firdes_rcos(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
void liquid_firdes_rrcos(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
void liquid_firdes_rkaiser(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
void liquid_firdes_arkaiser(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
float rkaiser_approximate_rho(unsigned int _m, float _beta);
void liquid_firdes_hM3(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
void liquid_firdes_gmsktx(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
void liquid_firdes_gmskrx(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
void liquid_firdes_fexp(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
void liquid_firdes_rfexp(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
void liquid_firdes_fsech(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
void liquid_firdes_rfsech(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
void liquid_firdes_farcsech(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
void liquid_firdes_rfarcsech(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h);
/* liquid.h:1635-1668 */
float liquid_filter_autocorr(float *_h, unsigned int _h_len, int _lag);
void liquid_filter_isi(float *_h, unsigned int _k, unsigned int _m, float *_rms, float *_max);
/* liquid.h:4396 */
float liquid_Qf(float _z);
/* windows, liquid.h:4425-4465 */
float kaiser(unsigned int _n, unsigned int _N, float _beta, float _mu);
float hamming(unsigned int _n, unsigned int _N);
float hann(unsigned int _n, unsigned int _N);
float blackmanharris(unsigned int _n, unsigned int _N);
float liquid_rcostaper_windowf(unsigned int _n, unsigned int _t, unsigned int _N);
float liquid_kbd(unsigned int _n, unsigned int _N, float _beta);
void liquid_kbd_window(unsigned int _n, float _beta, float *_w);

/* ------------------------------------------------------------------------ */
/* random helpers (liquid.h:6301-6315): test-signal generation on the host   */
/* ------------------------------------------------------------------------ */
float randf(void);
float randnf(void);
void awgn(float *_x, float _nstd);
void crandnf(liquid_float_complex *_y);
void cawgn(liquid_float_complex *_x, float _nstd);

/* ------------------------------------------------------------------------ */
/* window buffers (liquid.h:296-349): the last _n samples, contiguous,       */
/* oldest first.  A host container by contract (read() hands the caller a    */
/* host pointer); the streaming objects below keep their own history on the */
/* device and do not use it.                                                 */
/* ------------------------------------------------------------------------ */
#define LQMI_WINDOW_API(WINDOW, T)                                                              \
    typedef struct WINDOW##_s *WINDOW;                                                          \
    WINDOW WINDOW##_create(unsigned int _n);                                                    \
    WINDOW WINDOW##_recreate(WINDOW _q, unsigned int _n);                                       \
    void WINDOW##_destroy(WINDOW _q);                                                           \
    void WINDOW##_print(WINDOW _q);                                                             \
    void WINDOW##_debug_print(WINDOW _q);                                                       \
    void WINDOW##_clear(WINDOW _q);                                                             \
    void WINDOW##_read(WINDOW _q, T **_v);                                                      \
    void WINDOW##_index(WINDOW _q, unsigned int _i, T *_v);                                     \
    void WINDOW##_push(WINDOW _q, T _v);                                                        \
    void WINDOW##_write(WINDOW _q, T *_v, unsigned int _n);

LQMI_WINDOW_API(windowf, float)
LQMI_WINDOW_API(windowcf, liquid_float_complex)

/* ------------------------------------------------------------------------ */
/* dotprod (liquid.h:503-560): rrrf, crcf, cccf                              */
/* ------------------------------------------------------------------------ */
#define LQMI_DOTPROD_API(DOTPROD, TO, TC, TI)                                                   \
    typedef struct DOTPROD##_s *DOTPROD;                                                        \
    void DOTPROD##_run(TC *_h, TI *_x, unsigned int _n, TO *_y);                                \
    void DOTPROD##_run4(TC *_h, TI *_x, unsigned int _n, TO *_y);                               \
    DOTPROD DOTPROD##_create(TC *_v, unsigned int _n);                                          \
    DOTPROD DOTPROD##_recreate(DOTPROD _q, TC *_v, unsigned int _n);                            \
    void DOTPROD##_destroy(DOTPROD _q);                                                         \
    void DOTPROD##_print(DOTPROD _q);                                                           \
    void DOTPROD##_execute(DOTPROD _q, TI *_v, TO *_y);                                         \
    /* extension: Y[v] = dot(h, X[v*_n .. v*_n+_n)), host pointers */                          \
    void DOTPROD##_execute_batch(DOTPROD _q, TI *_X, unsigned long long _nvec, TO *_Y);         \
    /* extension: same on device pointers, asynchronous on the object's stream */               \
    void DOTPROD##_execute_batch_dev(DOTPROD _q, const TI *_dX, unsigned long long _nvec,       \
                                     TO *_dY);                                                  \
    void DOTPROD##_set_stream(DOTPROD _q, void *_hip_stream);                                   \
    void *DOTPROD##_get_stream(DOTPROD _q);

LQMI_DOTPROD_API(dotprod_rrrf, float, float, float)
LQMI_DOTPROD_API(dotprod_crcf, liquid_float_complex, float, liquid_float_complex)
LQMI_DOTPROD_API(dotprod_cccf, liquid_float_complex, liquid_float_complex, liquid_float_complex)

/* ------------------------------------------------------------------------ */
/* firfilt (liquid.h:1985-2090): rrrf, crcf, cccf                            */
/* ------------------------------------------------------------------------ */
#define LQMI_FIRFILT_API(FIRFILT, TO, TC, TI)                                                   \
    typedef struct FIRFILT##_s *FIRFILT;                                                        \
    FIRFILT FIRFILT##_create(TC *_h, unsigned int _n);                                          \
    FIRFILT FIRFILT##_create_kaiser(unsigned int _n, float _fc, float _As, float _mu);          \
    FIRFILT FIRFILT##_create_rect(unsigned int _n);                                             \
    FIRFILT FIRFILT##_create_rnyquist(int _type, unsigned int _k, unsigned int _m, float _beta, float _mu);\
    FIRFILT FIRFILT##_recreate(FIRFILT _q, TC *_h, unsigned int _n);                            \
    void FIRFILT##_destroy(FIRFILT _q);                                                         \
    void FIRFILT##_reset(FIRFILT _q);                                                           \
    void FIRFILT##_print(FIRFILT _q);                                                           \
    void FIRFILT##_set_scale(FIRFILT _q, TC _scale);                                            \
    void FIRFILT##_push(FIRFILT _q, TI _x);                                                     \
    void FIRFILT##_execute(FIRFILT _q, TO *_y);                                                 \
    void FIRFILT##_execute_block(FIRFILT _q, TI *_x, unsigned int _n, TO *_y);                  \
    unsigned int FIRFILT##_get_length(FIRFILT _q);                                              \
    void FIRFILT##_freqresponse(FIRFILT _q, float _fc, liquid_float_complex *_H);               \
    float FIRFILT##_groupdelay(FIRFILT _q, float _fc);                                          \
    /* extension: device pointers (x == y allowed), asynchronous on the object's stream */      \
    void FIRFILT##_execute_block_dev(FIRFILT _q, const TI *_dx, unsigned long long _n,          \
                                     TO *_dy);                                                  \
    void FIRFILT##_set_stream(FIRFILT _q, void *_hip_stream);                                   \
    void *FIRFILT##_get_stream(FIRFILT _q);                                                     \
    void FIRFILT##_synchronize(FIRFILT _q);

LQMI_FIRFILT_API(firfilt_rrrf, float, float, float)
LQMI_FIRFILT_API(firfilt_crcf, liquid_float_complex, float, liquid_float_complex)
LQMI_FIRFILT_API(firfilt_cccf, liquid_float_complex, liquid_float_complex, liquid_float_complex)

/* ------------------------------------------------------------------------ */
/* firdecim (liquid.h:2664-2735): rrrf, crcf, cccf                           */
/* ------------------------------------------------------------------------ */
#define LQMI_FIRDECIM_API(FIRDECIM, TO, TC, TI)                                                 \
    typedef struct FIRDECIM##_s *FIRDECIM;                                                      \
    FIRDECIM FIRDECIM##_create(unsigned int _M, TC *_h, unsigned int _h_len);                   \
    FIRDECIM FIRDECIM##_create_kaiser(unsigned int _M, unsigned int _m, float _As);             \
    FIRDECIM FIRDECIM##_create_prototype(int _type, unsigned int _M, unsigned int _m, float _beta, float _dt);\
    void FIRDECIM##_destroy(FIRDECIM _q);                                                       \
    void FIRDECIM##_print(FIRDECIM _q);                                                         \
    void FIRDECIM##_clear(FIRDECIM _q);                                                         \
    void FIRDECIM##_execute(FIRDECIM _q, TI *_x, TO *_y);                                       \
    void FIRDECIM##_execute_block(FIRDECIM _q, TI *_x, unsigned int _n, TO *_y);                \
    /* extension: _n = number of outputs; _dx holds _n*M samples (device) */                    \
    void FIRDECIM##_execute_block_dev(FIRDECIM _q, const TI *_dx, unsigned long long _n,        \
                                      TO *_dy);                                                 \
    void FIRDECIM##_set_stream(FIRDECIM _q, void *_hip_stream);

LQMI_FIRDECIM_API(firdecim_rrrf, float, float, float)
LQMI_FIRDECIM_API(firdecim_crcf, liquid_float_complex, float, liquid_float_complex)
LQMI_FIRDECIM_API(firdecim_cccf, liquid_float_complex, liquid_float_complex, liquid_float_complex)

/* ------------------------------------------------------------------------ */
/* firinterp (liquid.h:2496-2565): rrrf, crcf, cccf                          */
/* ------------------------------------------------------------------------ */
#define LQMI_FIRINTERP_API(FIRINTERP, TO, TC, TI)                                               \
    typedef struct FIRINTERP##_s *FIRINTERP;                                                    \
    FIRINTERP FIRINTERP##_create(unsigned int _M, TC *_h, unsigned int _h_len);                 \
    FIRINTERP FIRINTERP##_create_kaiser(unsigned int _M, unsigned int _m, float _As);           \
    FIRINTERP FIRINTERP##_create_prototype(int _type, unsigned int _M, unsigned int _m, float _beta, float _dt);\
    void FIRINTERP##_destroy(FIRINTERP _q);                                                     \
    void FIRINTERP##_print(FIRINTERP _q);                                                       \
    void FIRINTERP##_reset(FIRINTERP _q);                                                       \
    void FIRINTERP##_execute(FIRINTERP _q, TI _x, TO *_y);                                      \
    void FIRINTERP##_execute_block(FIRINTERP _q, TI *_x, unsigned int _n, TO *_y);              \
    /* extension: _n inputs -> _n*M outputs, device pointers */                                 \
    void FIRINTERP##_execute_block_dev(FIRINTERP _q, const TI *_dx, unsigned long long _n,      \
                                       TO *_dy);                                                \
    void FIRINTERP##_set_stream(FIRINTERP _q, void *_hip_stream);

LQMI_FIRINTERP_API(firinterp_rrrf, float, float, float)
LQMI_FIRINTERP_API(firinterp_crcf, liquid_float_complex, float, liquid_float_complex)
LQMI_FIRINTERP_API(firinterp_cccf, liquid_float_complex, liquid_float_complex, liquid_float_complex)

/* ------------------------------------------------------------------------ */
/* firpfb (liquid.h:2392-2486): rrrf, crcf, cccf                             */
/* ------------------------------------------------------------------------ */
#define LQMI_FIRPFB_API(FIRPFB, TO, TC, TI)                                                     \
    typedef struct FIRPFB##_s *FIRPFB;                                                          \
    FIRPFB FIRPFB##_create(unsigned int _M, TC *_h, unsigned int _h_len);                       \
    FIRPFB FIRPFB##_create_kaiser(unsigned int _M, unsigned int _m, float _fc, float _As);      \
    FIRPFB FIRPFB##_create_rnyquist(int _type, unsigned int _M, unsigned int _k, unsigned int _m, float _beta);\
    FIRPFB FIRPFB##_create_drnyquist(int _type, unsigned int _M, unsigned int _k, unsigned int _m, float _beta);\
    FIRPFB FIRPFB##_recreate(FIRPFB _q, unsigned int _M, TC *_h, unsigned int _h_len);          \
    void FIRPFB##_destroy(FIRPFB _q);                                                           \
    void FIRPFB##_print(FIRPFB _q);                                                             \
    void FIRPFB##_set_scale(FIRPFB _q, TC _g);                                                  \
    void FIRPFB##_reset(FIRPFB _q);                                                             \
    void FIRPFB##_push(FIRPFB _q, TI _x);                                                       \
    void FIRPFB##_execute(FIRPFB _q, unsigned int _i, TO *_y);                                  \
    /* extension: push each of _n inputs and evaluate every bank after it:                   */ \
    /* _y[t*M + i] = execute(i) after push(_x[t]); host / device pointers                    */ \
    void FIRPFB##_execute_block(FIRPFB _q, TI *_x, unsigned long long _n, TO *_y);              \
    void FIRPFB##_execute_block_dev(FIRPFB _q, const TI *_dx, unsigned long long _n, TO *_dy);  \
    void FIRPFB##_set_stream(FIRPFB _q, void *_hip_stream);

LQMI_FIRPFB_API(firpfb_rrrf, float, float, float)
LQMI_FIRPFB_API(firpfb_crcf, liquid_float_complex, float, liquid_float_complex)
LQMI_FIRPFB_API(firpfb_cccf, liquid_float_complex, liquid_float_complex, liquid_float_complex)

/* ------------------------------------------------------------------------ */
/* resamp (liquid.h:2938-3015): rrrf, crcf, cccf                            */
/* ------------------------------------------------------------------------ */
#define LQMI_RESAMP_API(RESAMP, T)                                                                  \
    typedef struct RESAMP##_s *RESAMP;                                                              \
    RESAMP RESAMP##_create(float _rate, unsigned int _m, float _fc, float _As, unsigned int _npfb);  \
    RESAMP RESAMP##_create_default(float _rate);                                                    \
    void RESAMP##_destroy(RESAMP _q);                                                               \
    void RESAMP##_print(RESAMP _q);                                                                 \
    void RESAMP##_reset(RESAMP _q);                                                                 \
    unsigned int RESAMP##_get_delay(RESAMP _q);                                                     \
    void RESAMP##_set_rate(RESAMP _q, float _rate);                                                 \
    void RESAMP##_adjust_rate(RESAMP _q, float _delta);                                             \
    void RESAMP##_execute(RESAMP _q, T _x, T *_y, unsigned int *_num_written);                      \
    void RESAMP##_execute_block(RESAMP _q, T *_x, unsigned int _nx, T *_y, unsigned int *_ny);      \
    /* extension: number of outputs the next _nx inputs will produce (size _y with it) */          \
    unsigned long long RESAMP##_num_output(RESAMP _q, unsigned long long _nx);                      \
    /* extension: device pointers, asynchronous on the object's stream; *_ny is                     \
     * known (and written) before the call returns */                                               \
    void RESAMP##_execute_block_dev(RESAMP _q, const T *_dx, unsigned long long _nx, T *_dy,         \
                                    unsigned long long *_ny);                                       \
    void RESAMP##_set_stream(RESAMP _q, void *_hip_stream);                                         \
    void RESAMP##_synchronize(RESAMP _q);

LQMI_RESAMP_API(resamp_rrrf, float)
LQMI_RESAMP_API(resamp_crcf, liquid_float_complex)
LQMI_RESAMP_API(resamp_cccf, liquid_float_complex)

/* ------------------------------------------------------------------------ */
/* fft (liquid.h:1113-1216): plans bind host arrays; the transform runs on   */
/* the GPU.  liquid_nextpow2: liquid.h (math), src/math/src/math.c:143       */
/* ------------------------------------------------------------------------ */
typedef enum {
    LIQUID_FFT_UNKNOWN = 0,
    LIQUID_FFT_FORWARD = +1,
    LIQUID_FFT_BACKWARD = -1,
    LIQUID_FFT_REDFT00 = 10,
    LIQUID_FFT_REDFT10 = 11,
    LIQUID_FFT_REDFT01 = 12,
    LIQUID_FFT_REDFT11 = 13,
    LIQUID_FFT_RODFT00 = 20,
    LIQUID_FFT_RODFT10 = 21,
    LIQUID_FFT_RODFT01 = 22,
    LIQUID_FFT_RODFT11 = 23,
    LIQUID_FFT_MDCT = 30,
    LIQUID_FFT_IMDCT = 31,
} liquid_fft_type;
typedef struct fftplan_s *fftplan;
fftplan fft_create_plan(unsigned int _n, liquid_float_complex *_x, liquid_float_complex *_y, int _dir, int _flags);
fftplan fft_create_plan_r2r_1d(unsigned int _n, float *_x, float *_y, int _type, int _flags);
void fft_destroy_plan(fftplan _p);
void fft_print_plan(fftplan _p);
void fft_execute(fftplan _p);
void fft_run(unsigned int _n, liquid_float_complex *_x, liquid_float_complex *_y, int _dir, int _flags);
void fft_r2r_1d_run(unsigned int _n, float *_x, float *_y, int _type, int _flags);
void fft_shift(liquid_float_complex *_x, unsigned int _n);
unsigned int liquid_nextpow2(unsigned int _x);
/* extension: _batch transforms of the plan's size/direction (contiguous);
 * host arrays or device pointers (asynchronous on the plan's stream) */
void fft_execute_batch(fftplan _p, const void *_x, void *_y, unsigned long long _batch);
void fft_execute_batch_dev(fftplan _p, const void *_dx, void *_dy, unsigned long long _batch);
void fft_set_stream(fftplan _p, void *_hip_stream);

/* ------------------------------------------------------------------------ */
/* spgram (liquid.h:1220-1290): spgramcf (complex in), spgramf (real in)     */
/* ------------------------------------------------------------------------ */
#define LQMI_SPGRAM_API(SPGRAM, TI)                                                                 \
    typedef struct SPGRAM##_s *SPGRAM;                                                              \
    SPGRAM SPGRAM##_create(unsigned int _nfft, float *_window, unsigned int _window_len);          \
    SPGRAM SPGRAM##_create_kaiser(unsigned int _nfft, unsigned int _window_len, float _beta);      \
    SPGRAM SPGRAM##_create_default(unsigned int _nfft);                                             \
    void SPGRAM##_destroy(SPGRAM _q);                                                               \
    void SPGRAM##_reset(SPGRAM _q);                                                                 \
    void SPGRAM##_push(SPGRAM _q, TI _x);                                                           \
    void SPGRAM##_write(SPGRAM _q, TI *_x, unsigned int _n);                                        \
    void SPGRAM##_execute(SPGRAM _q, liquid_float_complex *_X);                                     \
    void SPGRAM##_execute_psd(SPGRAM _q, float *_X);                                                \
    void SPGRAM##_accumulate_psd(SPGRAM _q, TI *_x, float _alpha, unsigned int _n);                 \
    void SPGRAM##_write_accumulation(SPGRAM _q, float *_x);                                         \
    void SPGRAM##_estimate_psd(SPGRAM _q, TI *_x, unsigned int _n, float *_psd);                    \
    /* extensions: device-resident input (and psd output), asynchronous */                          \
    void SPGRAM##_accumulate_psd_dev(SPGRAM _q, const TI *_dx, float _alpha, unsigned long long _n); \
    void SPGRAM##_estimate_psd_dev(SPGRAM _q, const TI *_dx, unsigned long long _n, float *_dpsd);  \
    void SPGRAM##_set_stream(SPGRAM _q, void *_hip_stream);                                         \
    void SPGRAM##_synchronize(SPGRAM _q);

LQMI_SPGRAM_API(spgramcf, liquid_float_complex)
LQMI_SPGRAM_API(spgramf, float)

/* ------------------------------------------------------------------------ */
/* resamp2 (liquid.h:2840-2925), msresamp2 (:3027-3090), msresamp (:3094-3140) */
/* ------------------------------------------------------------------------ */
/* liquid.h:3022-3025 */
typedef enum {
    LIQUID_RESAMP_INTERP = 0,
    LIQUID_RESAMP_DECIM,
} liquid_resamp_type;

/* extension: mode argument of resamp2_*_execute_block[_dev] */
enum {
    LQMI_RESAMP2_FILTER = 0,       /* n calls: x[n] -> y0[n] (low band), y1[n] (high band) */
    LQMI_RESAMP2_ANALYZER,         /* x[2n] -> y0[2n] */
    LQMI_RESAMP2_SYNTHESIZER,      /* x[2n] -> y0[2n] */
    LQMI_RESAMP2_DECIM,            /* x[2n] -> y0[n] */
    LQMI_RESAMP2_INTERP,           /* x[n]  -> y0[2n] */
};

#define LQMI_RESAMP2_API(RESAMP2, T)                                                                \
    typedef struct RESAMP2##_s *RESAMP2;                                                            \
    RESAMP2 RESAMP2##_create(unsigned int _m, float _f0, float _As);                                \
    RESAMP2 RESAMP2##_recreate(RESAMP2 _q, unsigned int _m, float _f0, float _As);                  \
    void RESAMP2##_destroy(RESAMP2 _q);                                                             \
    void RESAMP2##_print(RESAMP2 _q);                                                               \
    void RESAMP2##_clear(RESAMP2 _q);                                                               \
    unsigned int RESAMP2##_get_delay(RESAMP2 _q);                                                   \
    void RESAMP2##_filter_execute(RESAMP2 _q, T _x, T *_y0, T *_y1);                                \
    void RESAMP2##_analyzer_execute(RESAMP2 _q, T *_x, T *_y);                                      \
    void RESAMP2##_synthesizer_execute(RESAMP2 _q, T *_x, T *_y);                                   \
    void RESAMP2##_decim_execute(RESAMP2 _q, T *_x, T *_y);                                         \
    void RESAMP2##_interp_execute(RESAMP2 _q, T _x, T *_y);                                         \
    /* extension: _n consecutive calls of one mode (LQMI_RESAMP2_*); _y1 only for FILTER */         \
    void RESAMP2##_execute_block(RESAMP2 _q, int _mode, T *_x, unsigned long long _n, T *_y0, T *_y1); \
    void RESAMP2##_execute_block_dev(RESAMP2 _q, int _mode, const T *_dx, unsigned long long _n,    \
                                     T *_dy0, T *_dy1);                                             \
    void RESAMP2##_set_stream(RESAMP2 _q, void *_hip_stream);                                       \
    void RESAMP2##_synchronize(RESAMP2 _q);

LQMI_RESAMP2_API(resamp2_rrrf, float)
LQMI_RESAMP2_API(resamp2_crcf, liquid_float_complex)
LQMI_RESAMP2_API(resamp2_cccf, liquid_float_complex)

#define LQMI_MSRESAMP2_API(MSRESAMP2, T)                                                            \
    typedef struct MSRESAMP2##_s *MSRESAMP2;                                                        \
    MSRESAMP2 MSRESAMP2##_create(int _type, unsigned int _num_stages, float _fc, float _f0, float _As); \
    void MSRESAMP2##_destroy(MSRESAMP2 _q);                                                         \
    void MSRESAMP2##_print(MSRESAMP2 _q);                                                           \
    void MSRESAMP2##_reset(MSRESAMP2 _q);                                                           \
    float MSRESAMP2##_get_delay(MSRESAMP2 _q);                                                      \
    void MSRESAMP2##_execute(MSRESAMP2 _q, T *_x, T *_y);                                           \
    /* extension: _n consecutive calls (interp: 1 in, 2^s out; decim: 2^s in, 1 out) */            \
    void MSRESAMP2##_execute_block(MSRESAMP2 _q, T *_x, unsigned long long _n, T *_y);              \
    void MSRESAMP2##_execute_block_dev(MSRESAMP2 _q, const T *_dx, unsigned long long _n, T *_dy);  \
    void MSRESAMP2##_set_stream(MSRESAMP2 _q, void *_hip_stream);                                   \
    void MSRESAMP2##_synchronize(MSRESAMP2 _q);

LQMI_MSRESAMP2_API(msresamp2_rrrf, float)
LQMI_MSRESAMP2_API(msresamp2_crcf, liquid_float_complex)
LQMI_MSRESAMP2_API(msresamp2_cccf, liquid_float_complex)

#define LQMI_MSRESAMP_API(MSRESAMP, T)                                                              \
    typedef struct MSRESAMP##_s *MSRESAMP;                                                          \
    MSRESAMP MSRESAMP##_create(float _r, float _As);                                                \
    void MSRESAMP##_destroy(MSRESAMP _q);                                                           \
    void MSRESAMP##_print(MSRESAMP _q);                                                             \
    void MSRESAMP##_reset(MSRESAMP _q);                                                             \
    float MSRESAMP##_get_delay(MSRESAMP _q);                                                        \
    void MSRESAMP##_execute(MSRESAMP _q, T *_x, unsigned int _nx, T *_y, unsigned int *_ny);        \
    /* extension: outputs the next _nx inputs produce; device-pointer form */                       \
    unsigned long long MSRESAMP##_num_output(MSRESAMP _q, unsigned long long _nx);                  \
    void MSRESAMP##_execute_block_dev(MSRESAMP _q, const T *_dx, unsigned long long _nx, T *_dy,    \
                                      unsigned long long *_ny);                                     \
    void MSRESAMP##_set_stream(MSRESAMP _q, void *_hip_stream);                                     \
    void MSRESAMP##_synchronize(MSRESAMP _q);

LQMI_MSRESAMP_API(msresamp_rrrf, float)
LQMI_MSRESAMP_API(msresamp_crcf, liquid_float_complex)
LQMI_MSRESAMP_API(msresamp_cccf, liquid_float_complex)

/* ------------------------------------------------------------------------ */
/* fftfilt (liquid.h:2192-2240): rrrf, crcf, cccf                            */
/* ------------------------------------------------------------------------ */
#define LQMI_FFTFILT_API(FFTFILT, TO, TC, TI)                                                   \
    typedef struct FFTFILT##_s *FFTFILT;                                                        \
    FFTFILT FFTFILT##_create(TC *_h, unsigned int _h_len, unsigned int _n);                     \
    void FFTFILT##_destroy(FFTFILT _q);                                                         \
    void FFTFILT##_reset(FFTFILT _q);                                                           \
    void FFTFILT##_print(FFTFILT _q);                                                           \
    void FFTFILT##_set_scale(FFTFILT _q, TC _scale);                                            \
    void FFTFILT##_execute(FFTFILT _q, TI *_x, TO *_y);                                         \
    unsigned int FFTFILT##_get_length(FFTFILT _q);                                              \
    /* extension: arbitrary-length stream (any _n), host / device pointers */                   \
    void FFTFILT##_execute_block(FFTFILT _q, TI *_x, unsigned long long _n, TO *_y);            \
    void FFTFILT##_execute_block_dev(FFTFILT _q, const TI *_dx, unsigned long long _n,          \
                                     TO *_dy);                                                  \
    void FFTFILT##_set_stream(FFTFILT _q, void *_hip_stream);

LQMI_FFTFILT_API(fftfilt_rrrf, float, float, float)
LQMI_FFTFILT_API(fftfilt_crcf, liquid_float_complex, float, liquid_float_complex)
LQMI_FFTFILT_API(fftfilt_cccf, liquid_float_complex, liquid_float_complex, liquid_float_complex)

/* ------------------------------------------------------------------------ */
/* firpfbch (liquid.h:5667-5739): crcf, cccf                                 */
/* ------------------------------------------------------------------------ */
#define LQMI_FIRPFBCH_API(FIRPFBCH, TC)                                                             \
    typedef struct FIRPFBCH##_s *FIRPFBCH;                                                          \
    FIRPFBCH FIRPFBCH##_create(int _type, unsigned int _M, unsigned int _p, TC *_h);                \
    FIRPFBCH FIRPFBCH##_create_kaiser(int _type, unsigned int _M, unsigned int _m, float _As);      \
    FIRPFBCH FIRPFBCH##_create_rnyquist(int _type, unsigned int _M, unsigned int _m, float _beta,   \
                                        int _ftype);                                                \
    void FIRPFBCH##_destroy(FIRPFBCH _q);                                                           \
    void FIRPFBCH##_reset(FIRPFBCH _q);                                                             \
    void FIRPFBCH##_print(FIRPFBCH _q);                                                             \
    void FIRPFBCH##_synthesizer_execute(FIRPFBCH _q, liquid_float_complex *_x,                      \
                                        liquid_float_complex *_y);                                  \
    void FIRPFBCH##_analyzer_execute(FIRPFBCH _q, liquid_float_complex *_x,                         \
                                     liquid_float_complex *_y);                                     \
    /* extension: _nblocks consecutive M-sample blocks (analyzer or synthesizer) */                 \
    void FIRPFBCH##_execute_block(FIRPFBCH _q, liquid_float_complex *_x, unsigned long long _nblocks, \
                                  liquid_float_complex *_y);                                        \
    void FIRPFBCH##_execute_block_dev(FIRPFBCH _q, const liquid_float_complex *_dx,                 \
                                      unsigned long long _nblocks, liquid_float_complex *_dy);      \
    void FIRPFBCH##_set_stream(FIRPFBCH _q, void *_hip_stream);

LQMI_FIRPFBCH_API(firpfbch_crcf, float)
LQMI_FIRPFBCH_API(firpfbch_cccf, liquid_float_complex)

/* ------------------------------------------------------------------------ */
/* firpfbch2 (liquid.h:5754-5799): crcf                                      */
/* ------------------------------------------------------------------------ */
typedef struct firpfbch2_crcf_s *firpfbch2_crcf;
firpfbch2_crcf firpfbch2_crcf_create(int _type, unsigned int _M, unsigned int _m, float *_h);
firpfbch2_crcf firpfbch2_crcf_create_kaiser(int _type, unsigned int _M, unsigned int _m, float _As);
void firpfbch2_crcf_destroy(firpfbch2_crcf _q);
void firpfbch2_crcf_reset(firpfbch2_crcf _q);
void firpfbch2_crcf_print(firpfbch2_crcf _q);
void firpfbch2_crcf_execute(firpfbch2_crcf _q, liquid_float_complex *_x, liquid_float_complex *_y);
/* extension: _nblocks consecutive execute() calls.  analyzer: _x = _nblocks*M/2 inputs,
 * _y = _nblocks*M outputs; synthesizer: _nblocks*M in, _nblocks*M/2 out */
void firpfbch2_crcf_execute_block(firpfbch2_crcf _q, liquid_float_complex *_x,
                                  unsigned long long _nblocks, liquid_float_complex *_y);
void firpfbch2_crcf_execute_block_dev(firpfbch2_crcf _q, const liquid_float_complex *_dx,
                                      unsigned long long _nblocks, liquid_float_complex *_dy);
void firpfbch2_crcf_set_stream(firpfbch2_crcf _q, void *_hip_stream);
void *firpfbch2_crcf_get_stream(firpfbch2_crcf _q);
void firpfbch2_crcf_synchronize(firpfbch2_crcf _q);

/* ------------------------------------------------------------------------ */
/* runtime extensions                                                        */
/* ------------------------------------------------------------------------ */
/* device memory helpers for callers without their own HIP code */
void *liquid_mi355x_malloc(unsigned long long _bytes);
void liquid_mi355x_free(void *_p);
void liquid_mi355x_memcpy_h2d(void *_dst, const void *_src, unsigned long long _bytes);
void liquid_mi355x_memcpy_d2h(void *_dst, const void *_src, unsigned long long _bytes);
void liquid_mi355x_device_synchronize(void);
/* build identification (gfx target the kernels were compiled for) */
const char *liquid_mi355x_build_target(void);
/* Small-call mode (no reference counterpart).  1 (default): the
 * single-sample / single-vector entry points -- firfilt_*_execute after push,
 * dotprod_*_execute / _run / _run4, firdecim_*_execute, firinterp_*_execute,
 * resamp_*_execute, and fftfilt_*_execute when n * h_len <= 65536 -- compute
 * on the host (host/lq_small.c); every *_execute_block[_dev] call, the
 * channelizers, FFT plans and spgram run on the GPU.  0: every call runs on
 * the GPU.  The environment variable LQ_SMALL_CALLS=gpu sets 0 at load. */
void liquid_mi355x_set_small_calls(int _host);
int liquid_mi355x_get_small_calls(void);

#ifdef __cplusplus
}
#endif

#endif /* LIQUID_MI355X_H */
