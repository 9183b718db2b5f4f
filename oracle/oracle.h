/*
 * oracle.h -- CPU restatement of liquid-dsp's streaming filter/channelizer path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (liquid-dsp_amd/, include/)
 * may include, link or call this.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py load oracle/_build/liboracle.so, and only as the
 * checker / the timed CPU baseline, never as the thing measured or shipped.
 *
 * Parity status: the reference itself is NOT buildable in this image (every
 * source includes the autoconf-generated "config.h" through
 * include/liquid.internal.h:36; no autoconf here), so the oracle is pinned by
 * the reference's own golden vectors (tests/golden/ JSON files, extracted by
 * tests/golden/gen_golden.py) for dotprod / firfilt / firdecim / firinterp /
 * firpfb / fftfilt / fft, and by the reference's own property tests
 * (firpfbch analyzer == mixer+firfilt, firpfbch2 analysis->synthesis perfect
 * reconstruction, resamp rate) for the objects that ship no golden data.
 *
 * Every function cites the reference file:line it restates.
 * Complex data is C99 `float complex` (interleaved re,im; 8 bytes).
 */
#ifndef LIQUID_ORACLE_H
#define LIQUID_ORACLE_H

#include <complex.h>

typedef float complex orc_cf;

/* ---- filter design (src/filter/src/firdes.c:224-281, src/math/src/math*.c) - */
float        orc_kaiser_beta_As(float As);
float        orc_sincf(float x);
float        orc_lngammaf(float z);
float        orc_besseli0f(float z);
float        orc_kaiser(unsigned int n, unsigned int N, float beta, float mu);
void         orc_firdes_kaiser(unsigned int n, float fc, float As, float mu, float *h);
unsigned int orc_msb_index(unsigned int x);

/* ---- dot products (src/dotprod/src/dotprod.c:42-89) ---------------------- */
void orc_dotprod_rrrf_run4(const float  *h, const float  *x, unsigned int n, float  *y);
void orc_dotprod_crcf_run4(const float  *h, const orc_cf *x, unsigned int n, orc_cf *y);
void orc_dotprod_cccf_run4(const orc_cf *h, const orc_cf *x, unsigned int n, orc_cf *y);
/* batched: Y[v] = dot(h, X[v*n .. v*n+n)) -- the BASELINE config-2 workload   */
void orc_dotprod_rrrf_batch(const float  *h, const float  *X, unsigned int n, unsigned long nvec, float  *Y);
void orc_dotprod_crcf_batch(const float  *h, const orc_cf *X, unsigned int n, unsigned long nvec, orc_cf *Y);
void orc_dotprod_cccf_batch(const orc_cf *h, const orc_cf *X, unsigned int n, unsigned long nvec, orc_cf *Y);

/* ---- FFT (src/fft/src/fft_common.c; dir +1 forward e^-j, -1 backward e^+j) */
void orc_fft(unsigned int n, const orc_cf *x, orc_cf *y, int dir);

/* ---- streaming objects ---------------------------------------------------- */
/* type codes used by the generic objects */
enum { ORC_RRRF = 0, ORC_CRCF = 1, ORC_CCCF = 2 };

/* firfilt (src/filter/src/firfilt.c:62-359).  h/x/y are float (rrrf) or
 * orc_cf (crcf x/y, cccf h/x/y) according to `type`. */
typedef struct orc_firfilt_s *orc_firfilt;
orc_firfilt  orc_firfilt_create(int type, const void *h, unsigned int n);
void         orc_firfilt_destroy(orc_firfilt q);
void         orc_firfilt_reset(orc_firfilt q);
void         orc_firfilt_set_scale(orc_firfilt q, float scale_re, float scale_im);
void         orc_firfilt_push(orc_firfilt q, const void *x);
void         orc_firfilt_execute(orc_firfilt q, void *y);
void         orc_firfilt_execute_block(orc_firfilt q, const void *x, unsigned int n, void *y);

/* firdecim (src/filter/src/firdecim.c:47-223) */
typedef struct orc_firdecim_s *orc_firdecim;
orc_firdecim orc_firdecim_create(int type, unsigned int M, const void *h, unsigned int h_len);
orc_firdecim orc_firdecim_create_kaiser(unsigned int M, unsigned int m, float As);
void         orc_firdecim_destroy(orc_firdecim q);
void         orc_firdecim_clear(orc_firdecim q);
void         orc_firdecim_execute_block(orc_firdecim q, const void *x, unsigned int n, void *y);

/* firpfb (src/filter/src/firpfb.c:46-345) */
typedef struct orc_firpfb_s *orc_firpfb;
orc_firpfb   orc_firpfb_create(int type, unsigned int M, const void *h, unsigned int h_len);
void         orc_firpfb_destroy(orc_firpfb q);
void         orc_firpfb_reset(orc_firpfb q);
void         orc_firpfb_set_scale(orc_firpfb q, float scale);
void         orc_firpfb_push(orc_firpfb q, const void *x);
void         orc_firpfb_execute(orc_firpfb q, unsigned int i, void *y);

/* firinterp (src/filter/src/firinterp.c:43-215) */
typedef struct orc_firinterp_s *orc_firinterp;
orc_firinterp orc_firinterp_create(int type, unsigned int M, const void *h, unsigned int h_len);
orc_firinterp orc_firinterp_create_kaiser(unsigned int M, unsigned int m, float As);
void          orc_firinterp_destroy(orc_firinterp q);
void          orc_firinterp_reset(orc_firinterp q);
void          orc_firinterp_execute_block(orc_firinterp q, const void *x, unsigned int n, void *y);

/* resamp_crcf (src/filter/src/resamp.c:79-363) */
typedef struct orc_resamp_s *orc_resamp;
orc_resamp   orc_resamp_create(float rate, unsigned int m, float fc, float As, unsigned int npfb);
void         orc_resamp_destroy(orc_resamp q);
void         orc_resamp_reset(orc_resamp q);
void         orc_resamp_set_rate(orc_resamp q, float rate);
void         orc_resamp_adjust_rate(orc_resamp q, float delta);
void         orc_resamp_execute_block(orc_resamp q, const orc_cf *x, unsigned int nx,
                                      orc_cf *y, unsigned int *ny);
/* the data-independent schedule: for each output k, the filter index b (or
 * -1 for a BOUNDARY output), the float32 mu bits, and the input index */
unsigned long orc_resamp_schedule(float rate, unsigned int npfb, unsigned long nx,
                                  int *b, float *mu, unsigned int *in_idx, unsigned long cap);

/* fftfilt (src/filter/src/fftfilt.c:69-260) */
typedef struct orc_fftfilt_s *orc_fftfilt;
orc_fftfilt  orc_fftfilt_create(int type, const void *h, unsigned int h_len, unsigned int n);
void         orc_fftfilt_destroy(orc_fftfilt q);
void         orc_fftfilt_reset(orc_fftfilt q);
void         orc_fftfilt_set_scale(orc_fftfilt q, float scale);
void         orc_fftfilt_execute(orc_fftfilt q, const void *x, void *y);

/* firpfbch_crcf (src/multichannel/src/firpfbch.c:73-409) */
typedef struct orc_firpfbch_s *orc_firpfbch;
orc_firpfbch orc_firpfbch_create(int type, unsigned int M, unsigned int p, const float *h);
orc_firpfbch orc_firpfbch_create_kaiser(int type, unsigned int M, unsigned int m, float As);
void         orc_firpfbch_destroy(orc_firpfbch q);
void         orc_firpfbch_reset(orc_firpfbch q);
void         orc_firpfbch_analyzer_execute(orc_firpfbch q, const orc_cf *x, orc_cf *y);
void         orc_firpfbch_synthesizer_execute(orc_firpfbch q, const orc_cf *x, orc_cf *y);

/* firpfbch2_crcf (src/multichannel/src/firpfbch2.c:66-357) */
typedef struct orc_firpfbch2_s *orc_firpfbch2;
orc_firpfbch2 orc_firpfbch2_create(int type, unsigned int M, unsigned int m, const float *h);
orc_firpfbch2 orc_firpfbch2_create_kaiser(int type, unsigned int M, unsigned int m, float As);
void          orc_firpfbch2_destroy(orc_firpfbch2 q);
void          orc_firpfbch2_reset(orc_firpfbch2 q);
void          orc_firpfbch2_execute(orc_firpfbch2 q, const orc_cf *x, orc_cf *y);
/* run `nblocks` consecutive execute() calls (analyzer: M/2 in, M out each) */
void          orc_firpfbch2_execute_block(orc_firpfbch2 q, const orc_cf *x, unsigned int nblocks, orc_cf *y);
/* prototype used by create_kaiser (firpfbch2.c:135-172): 2*M*m+1 taps */
void          orc_firpfbch2_prototype(int type, unsigned int M, unsigned int m, float As, float *h);

/* resamp2 (src/filter/src/resamp2.c:46-360): half-band filter/resampler.
 * ctaps: complex taps (cccf: exp(j 2 pi t f0) modulation), else real (cos). */
typedef struct orc_resamp2_s *orc_resamp2;
orc_resamp2   orc_resamp2_create(int ctaps, unsigned int m, float f0, float As);
void          orc_resamp2_destroy(orc_resamp2 q);
void          orc_resamp2_clear(orc_resamp2 q);
void          orc_resamp2_filter_execute(orc_resamp2 q, orc_cf x, orc_cf *y0, orc_cf *y1);
void          orc_resamp2_analyzer_execute(orc_resamp2 q, const orc_cf *x, orc_cf *y);
void          orc_resamp2_synthesizer_execute(orc_resamp2 q, const orc_cf *x, orc_cf *y);
void          orc_resamp2_decim_execute(orc_resamp2 q, const orc_cf *x, orc_cf *y);
void          orc_resamp2_interp_execute(orc_resamp2 q, orc_cf x, orc_cf *y);
void          orc_resamp2_run(orc_resamp2 q, int mode, const orc_cf *x, unsigned int n, orc_cf *y0, orc_cf *y1);

/* msresamp2 (src/filter/src/msresamp2.c:66-354): type 0 interp, 1 decim */
typedef struct orc_msresamp2_s *orc_msresamp2;
orc_msresamp2 orc_msresamp2_create(int ctaps, int type, unsigned int num_stages, float fc, float f0, float As);
void          orc_msresamp2_destroy(orc_msresamp2 q);
void          orc_msresamp2_reset(orc_msresamp2 q);
/* interp: 1 in, 2^s out; decim: 2^s in, 1 out */
void          orc_msresamp2_execute(orc_msresamp2 q, const orc_cf *x, orc_cf *y);

/* msresamp (src/filter/src/msresamp.c:68-349) */
typedef struct orc_msresamp_s *orc_msresamp;
orc_msresamp  orc_msresamp_create(float rate, float As);
void          orc_msresamp_destroy(orc_msresamp q);
void          orc_msresamp_reset(orc_msresamp q);
void          orc_msresamp_execute(orc_msresamp q, const orc_cf *x, unsigned int nx, orc_cf *y, unsigned int *ny);

/* spgram (src/fft/src/spgram.c:41-286): real_in selects spgramf */
typedef struct orc_spgram_s *orc_spgram;
orc_spgram orc_spgram_create(int real_in, unsigned int nfft, const float *window, unsigned int W);
void       orc_spgram_destroy(orc_spgram q);
void       orc_spgram_reset(orc_spgram q);
void       orc_spgram_write(orc_spgram q, const void *x, unsigned int n);
void       orc_spgram_execute(orc_spgram q, orc_cf *X);
void       orc_spgram_execute_psd(orc_spgram q, float *X);
void       orc_spgram_accumulate_psd(orc_spgram q, const void *x, float alpha, unsigned int n);
void       orc_spgram_write_accumulation(orc_spgram q, float *x);
void       orc_spgram_estimate_psd(orc_spgram q, const void *x, unsigned int n, float *psd);

#endif