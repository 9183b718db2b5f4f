/*
 * firdes.c -- prototype filter design used by the *_create_rnyquist /
 * *_create_prototype constructors (create time, host, as in the reference).
 *
 * Restated from liquid-dsp 1.2.0:
 *   liquid_firdes_prototype           src/filter/src/firdes.c:290-370
 *   estimate_req_filter_{len,As,df}   src/filter/src/firdes.c:52-176
 *   liquid_filter_autocorr / _isi     src/filter/src/firdes.c:420-532
 *   liquid_firdes_rcos                src/filter/src/rcos.c:37-81
 *   liquid_firdes_{a,}rkaiser         src/filter/src/rkaiser.c:47-150, 160-214, 337-486
 *   fexp / fsech / farcsech (+root)   src/filter/src/fnyquist.c:41-345
 *   liquid_firdes_gmsk{tx,rx}         src/filter/src/gmsk.c:37-194
 *   liquid_firdes_hM3                 src/filter/src/hM3.c:41-127
 *   firdespm_run (band-pass)          src/filter/src/firdespm.c:97-700
 * The DFTs the reference runs through fft_run() on odd lengths are evaluated
 * directly here (double accumulation); results agree to float rounding.
 */
#include <complex.h>
#include <math.h>

#include "lq_host.h"

/* ----------------------------------------------------------------- estimates */
static float lq_len_kaiser(float df, float As)
{
    if (df > 0.5f || df <= 0.0f) LQ_FAIL("error: estimate_req_filter_len_Kaiser(), invalid bandwidth : %f\n", df);
    if (As <= 0.0f) LQ_FAIL("error: estimate_req_filter_len(), invalid stopband level : %f\n", As);
    return (As - 7.95f) / (14.26f * df);   /* firdes.c:163-176 */
}

unsigned int estimate_req_filter_len(float _df, float _As)
{
    if (_df > 0.5f || _df <= 0.0f) LQ_FAIL("error: estimate_req_filter_len(), invalid bandwidth : %f\n", _df);
    if (_As <= 0.0f) LQ_FAIL("error: estimate_req_filter_len(), invalid stopband level : %f\n", _As);
    return (unsigned int)lq_len_kaiser(_df, _As);
}

/* bisection on the Kaiser length estimate (20 halvings of [0.01, 200] dB) */
float estimate_req_filter_As(float _df, unsigned int _N)
{
    float lo = 0.01f, hi = 200.0f, As = 0.0f;
    for (int it = 0; it < 20; it++) {
        As = 0.5f * (hi + lo);
        if (lq_len_kaiser(_df, As) < (float)_N) lo = As;
        else hi = As;
    }
    return As;
}

float estimate_req_filter_df(float _As, unsigned int _N)
{
    float lo = 1e-3f, hi = 0.499f, df = 0.0f;
    for (int it = 0; it < 20; it++) {
        df = 0.5f * (hi + lo);
        if (lq_len_kaiser(df, _As) < (float)_N) hi = df;
        else lo = df;
    }
    return df;
}

float liquid_Qf(float _z) { return 0.5f * (1.0f - erff(_z * (float)M_SQRT1_2)); }

float liquid_filter_autocorr(float *_h, unsigned int _h_len, int _lag)
{
    unsigned int lag = (unsigned int)abs(_lag);
    if (lag >= _h_len) return 0.0f;
    float r = 0.0f;
    for (unsigned int i = lag; i < _h_len; i++) r += _h[i] * _h[i - lag];
    return r;
}

/* ISI of a root-Nyquist filter through its autocorrelation at symbol lags */
void liquid_filter_isi(float *_h, unsigned int _k, unsigned int _m, float *_rms, float *_max)
{
    const unsigned int n = 2 * _k * _m + 1;
    const float r0 = liquid_filter_autocorr(_h, n, 0);
    float acc = 0.0f, mx = 0.0f;
    for (unsigned int i = 1; i <= 2 * _m; i++) {
        const float e = fabsf(liquid_filter_autocorr(_h, n, (int)(i * _k)) / r0);
        acc += e * e;
        if (i == 1 || e > mx) mx = e;
    }
    *_rms = sqrtf(acc / (float)(2 * _m));
    *_max = mx;
}

static void lq_normalise_energy(float *h, unsigned int n, unsigned int k)
{
    float e2 = 0.0f;
    for (unsigned int i = 0; i < n; i++) e2 += h[i] * h[i];
    for (unsigned int i = 0; i < n; i++) h[i] *= sqrtf(k / e2);
}

static void lq_check_kmb(const char *who, unsigned int k, unsigned int kmin, unsigned int m, float beta)
{
    if (k < kmin) {
        if (kmin == 2) LQ_FAIL("error: %s(): k must be greater than 1\n", who);
        LQ_FAIL("error: %s(): k must be greater than 0\n", who);
    }
    if (m < 1) LQ_FAIL("error: %s(): m must be greater than 0\n", who);
    if (beta < 0.0f || beta > 1.0f) LQ_FAIL("error: %s(): beta must be in [0,1]\n", who);
}

/* ------------------------------------------------------------- raised cosine */
static float lq_sinc(float x)
{
    if (fabsf(x) < 0.01f) return cosf(M_PI * x / 2.0f) * cosf(M_PI * x / 4.0f) * cosf(M_PI * x / 8.0f);
    return sinf(M_PI * x) / (M_PI * x);
}

void liquid_firdes_rcos(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    lq_check_kmb("liquid_firdes_rcos", _k, 1, _m, _beta);
    const unsigned int n = 2 * _k * _m + 1;
    for (unsigned int i = 0; i < n; i++) {
        const float z = ((float)i + _dt) / (float)_k - (float)_m;
        const float den = 1 - 4.0f * _beta * _beta * z * z;
        if (fabsf(den) < 1e-3f) _h[i] = sinf(M_PI / (2.0 * _beta)) * _beta * 0.5f;   /* the limit at z = 1/(2 beta) */
        else _h[i] = cosf(_beta * M_PI * z) * lq_sinc(z) / den;
    }
}

/* ---------------------------------------------------------- root-Nyquist Kaiser */
float rkaiser_approximate_rho(unsigned int _m, float _beta)
{
    if (_m < 1) LQ_FAIL("error: rkaiser_approximate_rho(): m must be greater than 0\n");
    if (_beta < 0.0f || _beta > 1.0f) LQ_FAIL("error: rkaiser_approximate_rho(): beta must be in [0,1]\n");
    /* fitted quadratic-in-log(beta) coefficients per m (rkaiser.c:171-195) */
    static const float C[22][3] = {
        {0.75749731f, 0.06134303f, -0.08729663f}, {0.81151861f, 0.07437658f, -0.01427088f},
        {0.84249538f, 0.07684185f, -0.00536879f}, {0.86140782f, 0.07144126f, -0.00558652f},
        {0.87457740f, 0.06578694f, -0.00650447f}, {0.88438797f, 0.06074265f, -0.00736405f},
        {0.89216620f, 0.05669236f, -0.00791222f}, {0.89874983f, 0.05361696f, -0.00815301f},
        {0.90460032f, 0.05167952f, -0.00807893f}, {0.91034430f, 0.05130753f, -0.00746192f},
        {0.91587675f, 0.05180436f, -0.00670711f}, {0.92121875f, 0.05273801f, -0.00588351f},
        {0.92638195f, 0.05400764f, -0.00508452f}, {0.93123555f, 0.05516163f, -0.00437306f},
        {0.93564993f, 0.05596561f, -0.00388152f}, {0.93976742f, 0.05662274f, -0.00348280f},
        {0.94351703f, 0.05694120f, -0.00318821f}, {0.94557273f, 0.05227591f, -0.00400676f},
        {0.95001614f, 0.05681641f, -0.00300628f}, {0.95281708f, 0.05637607f, -0.00304790f},
        {0.95536256f, 0.05575880f, -0.00312988f}, {0.95754206f, 0.05426060f, -0.00385945f},
    };
    float c0, c1, c2;
    if (_m <= 22) {
        c0 = C[_m - 1][0];
        c1 = C[_m - 1][1];
        c2 = C[_m - 1][2];
    } else {
        c0 = 0.056873f * logf(_m + 1e-3f) + 0.781388f;
        c1 = 0.05426f;
        c2 = -0.00386f;
    }
    const float b = logf(_beta);
    float rho = c0 + c1 * b + c2 * b * b;
    return rho < 0.0f ? 0.0f : (rho > 1.0f ? 1.0f : rho);
}

/* Kaiser design for bandwidth adjustment rho, returns the RMS ISI (rkaiser.c:488-516) */
static float lq_rkaiser_isi(unsigned int k, unsigned int m, float beta, float dt, float rho, float *h)
{
    if (rho < 0.0f) fprintf(stderr, "warning: liquid_firdes_rkaiser_internal_isi(), rho < 0\n");
    else if (rho > 1.0f) fprintf(stderr, "warning: liquid_firdes_rkaiser_internal_isi(), rho > 1\n");
    const unsigned int n = 2 * k * m + 1;
    const float kf = (float)k;
    const float df = beta * rho / kf;
    const float As = estimate_req_filter_As(df, n);
    const float fc = 0.5f * (1 + beta * (1.0f - rho)) / kf;
    liquid_firdes_kaiser(n, fc, As, dt, h);
    float rms, mx;
    liquid_filter_isi(h, k, m, &rms, &mx);
    return rms;
}

static void lq_check_rkaiser(const char *who, unsigned int k, unsigned int m, float beta, float dt)
{
    if (k < 2) LQ_FAIL("error: %s(), k must be at least 2\n", who);
    if (m < 1) LQ_FAIL("error: %s(), m must be at least 1\n", who);
    if (beta <= 0.0f || beta >= 1.0f) LQ_FAIL("error: %s(), beta must be in (0,1)\n", who);
    if (dt < -1.0f || dt > 1.0f) LQ_FAIL("error: %s(), dt must be in [-1,1]\n", who);
}

/* quadratic search over rho minimising the ISI (rkaiser.c:337-486) */
void liquid_firdes_rkaiser(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    lq_check_rkaiser("liquid_firdes_rkaiser", _k, _m, _beta, _dt);
    const unsigned int n = 2 * _k * _m + 1;
    const float rho_hat = rkaiser_approximate_rho(_m, _beta);
    float x1 = rho_hat, rho_opt = rho_hat, y_opt = 0.0f, dx = 0.2f;
    for (unsigned int p = 0; p < 14; p++) {
        float x0 = x1 - dx, x2 = x1 + dx;
        if (x0 <= 0.0f) x0 = 0.01f;
        if (x2 >= 1.0f) x2 = 0.99f;
        const float y0 = lq_rkaiser_isi(_k, _m, _beta, _dt, x0, _h);
        const float y1 = lq_rkaiser_isi(_k, _m, _beta, _dt, x1, _h);
        const float y2 = lq_rkaiser_isi(_k, _m, _beta, _dt, x2, _h);
        if (p == 0 || y1 < y_opt) {
            rho_opt = x1;
            y_opt = y1;
        }
        /* vertex of the parabola through the three points */
        const double ta = y0 * (x1 * x1 - x2 * x2) + y1 * (x2 * x2 - x0 * x0) + y2 * (x0 * x0 - x1 * x1);
        const double tb = y0 * (x1 - x2) + y1 * (x2 - x0) + y2 * (x0 - x1);
        const float x_hat = 0.5f * ta / tb;
        if (x_hat < x0 || x_hat > x2) break;
        if (p > 3 && fabsf(x_hat - x1) < 1e-6f) break;
        x1 = x_hat;
        dx *= 0.5f;
    }
    lq_rkaiser_isi(_k, _m, _beta, _dt, rho_opt, _h);
    lq_normalise_energy(_h, n, _k);
}

/* closed-form rho estimate (rkaiser.c:84-150) */
void liquid_firdes_arkaiser(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    lq_check_rkaiser("liquid_firdes_arkaiser", _k, _m, _beta, _dt);
    const float c0 = 0.762886 + 0.067663 * logf(_m);
    const float c1 = 0.065515;
    const float c2 = logf(1 - 0.088 * powf(_m, -1.6));
    const float lb = logf(_beta);
    float rho = c0 + c1 * lb + c2 * lb * lb;
    if (rho <= 0.0f || rho >= 1.0f) rho = rkaiser_approximate_rho(_m, _beta);
    const unsigned int n = 2 * _k * _m + 1;
    const float kf = (float)_k;
    const float df = _beta * rho / kf;
    const float As = estimate_req_filter_As(df, n);
    const float fc = 0.5f * (1 + _beta * (1.0f - rho)) / kf;
    liquid_firdes_kaiser(n, fc, As, _dt, _h);
    lq_normalise_energy(_h, n, _k);
}

/* -------------------------------------------------- flipped Nyquist families */
enum { LQ_FN_EXP, LQ_FN_SECH, LQ_FN_ARCSECH };

static float lq_asechf(float z)
{
    if (z <= 0.0f || z > 1.0f) {
        fprintf(stderr, "warning: liquid_asechf(), input out of range\n");
        return 0.0f;
    }
    const float zi = 1.0f / z;
    return logf(sqrtf(zi - 1.0f) * sqrtf(zi + 1.0f) + zi);
}

/* sampled frequency response on h_len bins (fnyquist.c:144-345) */
static void lq_fnyquist_H(int fam, unsigned int k, unsigned int m, float beta, float *H)
{
    const unsigned int n = 2 * k * m + 1;
    const float f0 = 0.5f * (1.0f - beta) / (float)k;
    const float f1 = 0.5f * (1.0f) / (float)k;
    const float f2 = 0.5f * (1.0f + beta) / (float)k;
    const float B = 0.5f / (float)k;
    const float gamma = fam == LQ_FN_EXP ? logf(2.0f) / (beta * B) : logf(sqrtf(3.0f) + 2.0f) / (beta * B);
    const float zeta = 1.0f / (2.0f * beta * B);
    for (unsigned int i = 0; i < n; i++) {
        float f = (float)i / (float)n;
        if (f > 0.5f) f = f - 1.0f;
        f = fabsf(f);
        float v;
        if (f < f0) {
            v = 1.0f;
        } else if (f > f0 && f < f2) {
            const int lower = f < f1;
            switch (fam) {
            case LQ_FN_EXP:
                v = lower ? expf(gamma * (B * (1 - beta) - f)) : 1.0f - expf(gamma * (f - (1 + beta) * B));
                break;
            case LQ_FN_SECH:
                v = lower ? 1.0f / coshf(gamma * (f - B * (1 - beta)))
                          : 1.0f - 1.0f / coshf(gamma * (B * (1 + beta) - f));
                break;
            default:
                v = lower ? 1.0f - (zeta / gamma) * lq_asechf(zeta * (B * (1 + beta) - f))
                          : (zeta / gamma) * lq_asechf(zeta * (f - B * (1 - beta)));
            }
        } else {
            v = 0.0f;
        }
        H[i] = v;
    }
}

/* y[t] = sum_i X[i] exp(+-2 pi j i t / n): the reference's fft_run on odd n */
static void lq_dft(const float complex *X, float complex *y, unsigned int n, int backward)
{
    const double s = backward ? 2.0 * M_PI : -2.0 * M_PI;
    for (unsigned int t = 0; t < n; t++) {
        double re = 0.0, im = 0.0;
        for (unsigned int i = 0; i < n; i++) {
            const double a = s * (double)(((unsigned long long)i * t) % n) / (double)n;
            const double xr = crealf(X[i]), xi = cimagf(X[i]);
            re += xr * cos(a) - xi * sin(a);
            im += xr * sin(a) + xi * cos(a);
        }
        y[t] = (float)re + (float)im * I;
    }
}

static void lq_fnyquist(int fam, int root, unsigned int k, unsigned int m, float beta, float *h)
{
    lq_check_kmb("liquid_firdes_fnyquist", k, 1, m, beta);
    const unsigned int n = 2 * k * m + 1;
    float *Hp = (float *)lq_xmalloc(n * sizeof(float));
    float complex *H = (float complex *)lq_xmalloc(n * sizeof(float complex));
    float complex *t = (float complex *)lq_xmalloc(n * sizeof(float complex));
    lq_fnyquist_H(fam, k, m, beta, Hp);
    for (unsigned int i = 0; i < n; i++) H[i] = root ? sqrtf(Hp[i]) : Hp[i];
    lq_dft(H, t, n, 1);
    for (unsigned int i = 0; i < n; i++) h[i] = crealf(t[(i + k * m + 1) % n]) * (float)k / (float)n;
    free(Hp);
    free(H);
    free(t);
}

void liquid_firdes_fexp(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    lq_fnyquist(LQ_FN_EXP, 0, _k, _m, _beta, _h);
}
void liquid_firdes_rfexp(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    lq_fnyquist(LQ_FN_EXP, 1, _k, _m, _beta, _h);
}
void liquid_firdes_fsech(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    lq_fnyquist(LQ_FN_SECH, 0, _k, _m, _beta, _h);
}
void liquid_firdes_rfsech(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    lq_fnyquist(LQ_FN_SECH, 1, _k, _m, _beta, _h);
}
void liquid_firdes_farcsech(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    lq_fnyquist(LQ_FN_ARCSECH, 0, _k, _m, _beta, _h);
}
void liquid_firdes_rfarcsech(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    lq_fnyquist(LQ_FN_ARCSECH, 1, _k, _m, _beta, _h);
}

/* ----------------------------------------------------------------------- GMSK */
void liquid_firdes_gmsktx(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    lq_check_kmb("liquid_firdes_gmsktx", _k, 1, _m, _beta);
    const unsigned int n = 2 * _k * _m + 1;
    const float c0 = 1.0f / sqrtf(logf(2.0f));
    /* Gaussian-filtered rectangular pulse: difference of Q functions */
    for (unsigned int i = 0; i < n; i++) {
        const float t = (float)i / (float)(_k) - (float)(_m) + _dt;
        _h[i] = liquid_Qf(2 * M_PI * _beta * (t - 0.5f) * c0) - liquid_Qf(2 * M_PI * _beta * (t + 0.5f) * c0);
    }
    float e = 0.0f;
    for (unsigned int i = 0; i < n; i++) e += _h[i];
    for (unsigned int i = 0; i < n; i++) _h[i] *= M_PI / (2.0f * e);
    for (unsigned int i = 0; i < n; i++) _h[i] *= (float)_k;
}

/* receive filter: spectral ratio of a Kaiser Nyquist prototype to the
 * transmit pulse, shaped by a Kaiser gain response (gmsk.c:99-194) */
void liquid_firdes_gmskrx(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    lq_check_kmb("liquid_firdes_gmskrx", _k, 1, _m, _beta);
    const unsigned int k = _k, m = _m, n = 2 * k * m + 1;
    const float delta = 1e-3f;
    float *ht = (float *)lq_xmalloc(n * sizeof(float));
    float *hp = (float *)lq_xmalloc(n * sizeof(float));
    float *gp = (float *)lq_xmalloc(n * sizeof(float));
    float complex *a = (float complex *)lq_xmalloc(n * sizeof(float complex));
    float complex *Hp = (float complex *)lq_xmalloc(n * sizeof(float complex));
    float complex *Gp = (float complex *)lq_xmalloc(n * sizeof(float complex));
    float complex *Ht = (float complex *)lq_xmalloc(n * sizeof(float complex));
    liquid_firdes_gmsktx(k, m, _beta, 0.0f, ht);
    liquid_firdes_prototype(LIQUID_FIRFILT_KAISER, k, m, _beta, 0.0f, hp);
    liquid_firdes_kaiser(n, (0.7f + 0.1 * _beta) / (float)k, 60.0f, 0.0f, gp);
    for (unsigned int i = 0; i < n; i++) a[i] = hp[(i + k * m) % n];
    lq_dft(a, Hp, n, 0);
    for (unsigned int i = 0; i < n; i++) a[i] = gp[(i + k * m) % n];
    lq_dft(a, Gp, n, 0);
    for (unsigned int i = 0; i < n; i++) a[i] = ht[(i + k * m) % n];
    lq_dft(a, Ht, n, 0);
    float ht_min = 0.0f, hp_min = 0.0f, gp_min = 0.0f;
    for (unsigned int i = 0; i < n; i++) {
        if (i == 0 || crealf(Ht[i]) < ht_min) ht_min = crealf(Ht[i]);
        if (i == 0 || crealf(Hp[i]) < hp_min) hp_min = crealf(Hp[i]);
        if (i == 0 || crealf(Gp[i]) < gp_min) gp_min = crealf(Gp[i]);
    }
    for (unsigned int i = 0; i < n; i++) {
        float complex v = crealf(Hp[i] - hp_min + delta) / crealf(Ht[i] - ht_min + delta);
        v *= crealf(Gp[i] - gp_min) / crealf(Gp[0]);
        a[i] = v;
    }
    lq_dft(a, Hp, n, 1);
    for (unsigned int i = 0; i < n; i++) _h[i] = crealf(Hp[(i + k * m + 1) % n]) / (float)(k * n) * _k * _k;
    free(ht);
    free(hp);
    free(gp);
    free(a);
    free(Hp);
    free(Gp);
    free(Ht);
}

/* ------------------------------------------------------ Parks-McClellan (Remez) */
typedef struct {
    unsigned int h_len, s, r, nb, grid;
    double *F, *D, *W, *E, *x, *alpha, *c, rho;
    unsigned int *iext, nexch;
} lq_pm;

/* barycentric Lagrange weights, normalised by the first (poly.lagrange.c:104-124) */
static void lq_bary_fit(const double *x, unsigned int n, double *w)
{
    for (unsigned int j = 0; j < n; j++) {
        double p = 1.0;
        for (unsigned int k = 0; k < n; k++)
            if (k != j) p *= x[j] - x[k];
        w[j] = 1.0 / p;
    }
    const double w0 = w[0];
    for (unsigned int j = 0; j < n; j++) w[j] /= w0;
}

static double lq_bary_eval(const double *x, const double *y, const double *w, double x0, unsigned int n)
{
    double num = 0.0, den = 0.0;
    for (unsigned int j = 0; j < n; j++) {
        const double g = x0 - x[j];
        if (fabs(g) < 1e-6f) return y[j];
        num += w[j] * y[j] / g;
        den += w[j] / g;
    }
    return num / den;
}

/* alternation-point interpolant and deviation rho (firdespm.c:440-500) */
static void lq_pm_interp(lq_pm *q)
{
    const unsigned int n = q->r + 1;
    for (unsigned int i = 0; i < n; i++) q->x[i] = cos(2 * M_PI * q->F[q->iext[i]]);
    lq_bary_fit(q->x, n, q->alpha);
    double t0 = 0.0, t1 = 0.0;
    for (unsigned int i = 0; i < n; i++) {
        t0 += q->alpha[i] * q->D[q->iext[i]];
        t1 += q->alpha[i] / q->W[q->iext[i]] * (i % 2 ? -1.0 : 1.0);
    }
    q->rho = t0 / t1;
    for (unsigned int i = 0; i < n; i++) q->c[i] = q->D[q->iext[i]] - (i % 2 ? -1 : 1) * q->rho / q->W[q->iext[i]];
}

/* new extremal set: local extrema of the weighted error, surplus removed
 * keeping sign alternation (firdespm.c:520-640) */
static void lq_pm_search(lq_pm *q)
{
    const unsigned int nmax = 2 * q->r + 2 * q->nb;
    unsigned int *f = (unsigned int *)lq_xmalloc((nmax + 1) * sizeof(unsigned int));
    unsigned int nf = 0;
    const double *E = q->E;
    f[nf++] = 0;
    for (unsigned int i = 1; i + 1 < q->grid; i++) {
        if ((E[i] >= 0.0 && E[i - 1] <= E[i] && E[i + 1] <= E[i]) ||
            (E[i] < 0.0 && E[i - 1] >= E[i] && E[i + 1] >= E[i])) {
            if (nf >= nmax) LQ_FAIL("error: firdespm_iext_search(), too many extremal frequencies\n");
            f[nf++] = i;
        }
    }
    if (nf >= nmax) LQ_FAIL("error: firdespm_iext_search(), too many extremal frequencies\n");
    f[nf++] = q->grid - 1;
    if (nf < q->r + 1) {
        q->nexch = 0;
        free(f);
        return;
    }
    unsigned int extra = nf - q->r - 1;
    while (extra) {
        int sign = E[f[0]] > 0.0;
        unsigned int imin = 0;
        int alternating = 1;
        for (unsigned int i = 1; i < nf; i++) {
            if (fabs(E[f[i]]) < fabs(E[f[imin]])) imin = i;
            if (sign && E[f[i]] < 0.0) {
                sign = 0;
            } else if (!sign && E[f[i]] >= 0.0) {
                sign = 1;
            } else {
                imin = fabs(E[f[i]]) < fabs(E[f[i - 1]]) ? i : i - 1;
                alternating = 0;
                break;
            }
        }
        if (alternating && extra == 1) imin = fabs(E[f[0]]) < fabs(E[f[nf - 1]]) ? 0 : nf - 1;
        for (unsigned int i = imin; i + 1 < nf; i++) f[i] = f[i + 1];
        extra--;
        nf--;
    }
    q->nexch = 0;
    for (unsigned int i = 0; i < q->r + 1; i++) q->nexch += q->iext[i] == f[i] ? 0 : 1;
    memcpy(q->iext, f, (q->r + 1) * sizeof(unsigned int));
    free(f);
}

void firdespm_run(unsigned int _h_len, unsigned int _num_bands, float *_bands, float *_des, float *_weights,
                  liquid_firdespm_wtype *_wtype, liquid_firdespm_btype _btype, float *_h)
{
    int ok = 1, wok = 1;
    for (unsigned int i = 0; i < 2 * _num_bands; i++) ok &= _bands[i] >= 0.0 && _bands[i] <= 0.5;
    for (unsigned int i = 1; i < 2 * _num_bands; i++) ok &= _bands[i] >= _bands[i - 1];
    for (unsigned int i = 0; _weights && i < _num_bands; i++) wok &= _weights[i] > 0;
    if (!ok) LQ_FAIL("error: firdespm_create(), invalid bands\n");
    if (!wok) LQ_FAIL("error: firdespm_create(), invalid weights (must be positive)\n");
    if (_num_bands == 0) LQ_FAIL("error: firdespm_create(), number of bands must be > 0\n");
    if (_btype != LIQUID_FIRDESPM_BANDPASS)
        LQ_FAIL("error: firdespm_run(), only LIQUID_FIRDESPM_BANDPASS designs are provided by this build\n");
    lq_pm q;
    memset(&q, 0, sizeof(q));
    q.h_len = _h_len;
    q.s = _h_len % 2;
    q.r = (_h_len - q.s) / 2 + q.s;
    q.nb = _num_bands;
    /* dense grid: 20 points per approximating function (firdespm.c:196-210, 330-410) */
    const double df = 0.5 / (20.0 * q.r);
    unsigned int cap = 0;
    for (unsigned int i = 0; i < _num_bands; i++) cap += (unsigned int)(((double)_bands[2 * i + 1] - _bands[2 * i]) / df + 1.0);
    cap += _num_bands;
    q.F = (double *)lq_xmalloc(cap * sizeof(double));
    q.D = (double *)lq_xmalloc(cap * sizeof(double));
    q.W = (double *)lq_xmalloc(cap * sizeof(double));
    q.E = (double *)lq_xmalloc(cap * sizeof(double));
    q.x = (double *)lq_xmalloc((q.r + 1) * sizeof(double));
    q.alpha = (double *)lq_xmalloc((q.r + 1) * sizeof(double));
    q.c = (double *)lq_xmalloc((q.r + 1) * sizeof(double));
    q.iext = (unsigned int *)lq_xmalloc((q.r + 1) * sizeof(unsigned int));
    unsigned int g = 0;
    for (unsigned int i = 0; i < _num_bands; i++) {
        const double f0 = _bands[2 * i], f1 = _bands[2 * i + 1];
        unsigned int np = (unsigned int)((f1 - f0) / df + 0.5);
        if (np < 1) np = 1;
        const liquid_firdespm_wtype wt = _wtype ? _wtype[i] : LIQUID_FIRDESPM_FLATWEIGHT;
        for (unsigned int j = 0; j < np && g < cap; j++) {
            q.F[g] = f0 + j * df;
            q.D[g] = _des[i];
            double fw = 1.0f;
            if (wt == LIQUID_FIRDESPM_EXPWEIGHT) fw = expf(2.0f * j * df);
            else if (wt == LIQUID_FIRDESPM_LINWEIGHT) fw = 1.0f + 2.7f * j * df;
            else if (wt != LIQUID_FIRDESPM_FLATWEIGHT) LQ_FAIL("error: firdespm_init_grid(), invalid weighting specifyier: %d\n", wt);
            q.W[g] = (_weights ? _weights[i] : 1.0f) * fw;
            g++;
        }
        q.F[g - 1] = f1;
    }
    q.grid = g;
    if (q.s == 0) /* even length: H(f) = cos(pi f) P(f) */
        for (unsigned int i = 0; i < q.grid; i++) {
            q.D[i] /= cos(M_PI * q.F[i]);
            q.W[i] *= cos(M_PI * q.F[i]);
        }
    for (unsigned int i = 0; i < q.r + 1; i++) q.iext[i] = (i * (q.grid - 1)) / q.r;
    for (unsigned int it = 0; it < 40; it++) {
        lq_pm_interp(&q);
        for (unsigned int i = 0; i < q.grid; i++) {
            const double H = lq_bary_eval(q.x, q.c, q.alpha, cos(2 * M_PI * q.F[i]), q.r + 1);
            q.E[i] = q.W[i] * (q.D[i] - H);
        }
        lq_pm_search(&q);
        if (q.nexch == 0) break;
        double emin = 0.0, emax = 0.0;
        for (unsigned int i = 0; i < q.r + 1; i++) {
            const double e = fabs(q.E[q.iext[i]]);
            if (i == 0 || e < emin) emin = e;
            if (i == 0 || e > emax) emax = e;
        }
        if ((emax - emin) / emax < 1e-3f) break;
    }
    /* taps from the frequency samples (firdespm.c:660-700) */
    lq_pm_interp(&q);
    const unsigned int p = q.r - q.s + 1;
    double *G = (double *)lq_xmalloc(p * sizeof(double));
    for (unsigned int i = 0; i < p; i++) {
        const double f = (double)i / (double)q.h_len;
        const double cf = lq_bary_eval(q.x, q.c, q.alpha, cos(2 * M_PI * f), q.r + 1);
        G[i] = cf * (q.s == 1 ? 1.0 : cos(M_PI * i / q.h_len));
    }
    for (unsigned int i = 0; i < q.h_len; i++) {
        double v = G[0];
        const double f = ((double)i - (double)(p - 1) + 0.5 * (1 - q.s)) / (double)q.h_len;
        for (unsigned int j = 1; j < q.r; j++) v += 2.0 * G[j] * cos(2 * M_PI * f * j);
        _h[i] = v / (double)q.h_len;
    }
    free(G);
    free(q.F);
    free(q.D);
    free(q.W);
    free(q.E);
    free(q.x);
    free(q.alpha);
    free(q.c);
    free(q.iext);
}

/* harris-Moerder-3: PM design with the pass-band edge walked in until the
 * ISI stops improving (hM3.c:41-127) */
void liquid_firdes_hM3(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    lq_check_kmb("liquid_firdes_hM3", _k, 2, _m, _beta);
    const unsigned int n = 2 * _k * _m + 1;
    const float fc = 1.0 / (float)(2 * _k);
    const float fs = fc * (1.0 + _beta);
    float bands[6] = {0.0f, fc * (1.0 - _beta), fc, fc, fs, 0.5f};
    float des[3] = {1.0f, 1.0f / sqrtf(2.0f), 0.0f};
    float w[3] = {1.0f, 1.0f, 1.0f};
    liquid_firdespm_wtype wt[3] = {LIQUID_FIRDESPM_FLATWEIGHT, LIQUID_FIRDESPM_FLATWEIGHT, LIQUID_FIRDESPM_EXPWEIGHT};
    float *h = (float *)lq_xmalloc(n * sizeof(float));
    firdespm_run(n, 3, bands, des, w, wt, LIQUID_FIRDESPM_BANDPASS, h);
    memcpy(_h, h, n * sizeof(float));
    float rms, mx;
    liquid_filter_isi(h, _k, _m, &rms, &mx);
    float best = rms;
    for (unsigned int p = 0; p < 100; p++) {
        bands[1] = fc * (1.0 - _beta * p / (float)(100));
        firdespm_run(n, 3, bands, des, w, wt, LIQUID_FIRDESPM_BANDPASS, h);
        liquid_filter_isi(h, _k, _m, &rms, &mx);
        if (rms > best) break;
        best = rms;
        memcpy(_h, h, n * sizeof(float));
    }
    free(h);
    lq_normalise_energy(_h, n, _k);
}

/* ------------------------------------------------------------------ prototype */
void liquid_firdes_prototype(liquid_firfilt_type _type, unsigned int _k, unsigned int _m, float _beta, float _dt,
                             float *_h)
{
    const unsigned int n = 2 * _k * _m + 1;
    const float fc = 0.5f / (float)_k;
    const float df = _beta / (float)_k;
    switch (_type) {
    case LIQUID_FIRFILT_KAISER:
        liquid_firdes_kaiser(n, fc, estimate_req_filter_As(df, n), _dt, _h);
        break;
    case LIQUID_FIRFILT_PM: {
        /* the reference ignores _dt here too (firdes.c:320-323) */
        float bands[6] = {0.0f, fc - 0.5f * df, fc, fc, fc + 0.5f * df, 0.5f};
        float des[3] = {(float)_k, 0.5f * _k, 0.0f};
        float w[3] = {1.0f, 1.0f, 1.0f};
        liquid_firdespm_wtype wt[3] = {LIQUID_FIRDESPM_FLATWEIGHT, LIQUID_FIRDESPM_FLATWEIGHT,
                                       LIQUID_FIRDESPM_FLATWEIGHT};
        firdespm_run(n, 3, bands, des, w, wt, LIQUID_FIRDESPM_BANDPASS, _h);
        break;
    }
    case LIQUID_FIRFILT_RCOS: liquid_firdes_rcos(_k, _m, _beta, _dt, _h); break;
    case LIQUID_FIRFILT_FEXP: liquid_firdes_fexp(_k, _m, _beta, _dt, _h); break;
    case LIQUID_FIRFILT_FSECH: liquid_firdes_fsech(_k, _m, _beta, _dt, _h); break;
    case LIQUID_FIRFILT_FARCSECH: liquid_firdes_farcsech(_k, _m, _beta, _dt, _h); break;
    case LIQUID_FIRFILT_ARKAISER: liquid_firdes_arkaiser(_k, _m, _beta, _dt, _h); break;
    case LIQUID_FIRFILT_RKAISER: liquid_firdes_rkaiser(_k, _m, _beta, _dt, _h); break;
    case LIQUID_FIRFILT_RRC: liquid_firdes_rrcos(_k, _m, _beta, _dt, _h); break;
    case LIQUID_FIRFILT_hM3: liquid_firdes_hM3(_k, _m, _beta, _dt, _h); break;
    case LIQUID_FIRFILT_GMSKTX: liquid_firdes_gmsktx(_k, _m, _beta, _dt, _h); break;
    case LIQUID_FIRFILT_GMSKRX: liquid_firdes_gmskrx(_k, _m, _beta, _dt, _h); break;
    case LIQUID_FIRFILT_RFEXP: liquid_firdes_rfexp(_k, _m, _beta, _dt, _h); break;
    case LIQUID_FIRFILT_RFSECH: liquid_firdes_rfsech(_k, _m, _beta, _dt, _h); break;
    case LIQUID_FIRFILT_RFARCSECH: liquid_firdes_rfarcsech(_k, _m, _beta, _dt, _h); break;
    default:
        LQ_FAIL("error: liquid_firdes_prototype(), invalid root-Nyquist filter type '%d'\n", _type);
    }
}

int liquid_getopt_str2firfilt(const char *_str)
{
    static const char *names[] = {"kaiser", "pm", "rcos", "fexp", "fsech", "farcsech", "arkaiser", "rkaiser",
                                  "rrcos", "hM3", "gmsktx", "gmskrx", "rfexp", "rfsech", "rfarcsech"};
    for (unsigned int i = 0; i < sizeof(names) / sizeof(names[0]); i++)
        if (strcmp(_str, names[i]) == 0) return (int)i + 1;
    return LIQUID_FIRFILT_UNKNOWN;
}
