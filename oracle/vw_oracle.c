/*
 * vw_oracle.c -- CPU restatement of VectorWave's MODWT / SWT hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in vectorwave_amd/ links, loads or calls
 * this file.  It is used by tests/ (as the parity checker), by
 * __graft_entry__.smoke() (as the checker) and by bench.py's cpu_baseline leg.
 *
 * Every function restates one Java loop of the reference (MorphIQ-Labs/
 * VectorWave, mounted read-only at /root/reference) and keeps its exact
 * IEEE-754 binary64 operation order: separate multiply and add (Java has no
 * FMA contraction), taps visited in ascending order, zero taps of the
 * upsampled filters multiplied and added exactly as the Java loops do.  Build
 * with `-O2 -ffp-contract=off -fno-fast-math` (oracle/Makefile) so the result
 * is bit-identical to the JVM's.
 *
 * Path prefixes in citations:
 *   core/ = vectorwave-core/src/main/java/com/morphiqlabs/wavelet/
 *   ext/  = vectorwave-extensions/src/main/java/com/morphiqlabs/wavelet/
 *   fft/  = vectorwave-fft/src/main/java/com/morphiqlabs/wavelet/fft/
 *
 * Pinned by: tests/test_oracle_golden.py (known answers of the reference's
 * JUnit tests, its P&W restatements, round-trip/energy tolerances and the
 * SYMMETRIC NRMSE baseline fixture).
 *
 * Integer arithmetic follows Java `int` semantics: C99 `/` and `%` truncate
 * toward zero exactly like Java's.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* Boundary codes (same numbering as include/vectorwave_amd.h). */
enum { VWO_PERIODIC = 0, VWO_SYMMETRIC = 1, VWO_ZERO_PADDING = 2 };

/* Status codes (same numbering as include/vectorwave_amd.h). */
enum {
    VWO_OK = 0, VWO_ERR_NULL = 1, VWO_ERR_EMPTY = 2, VWO_ERR_NONFINITE = 3,
    VWO_ERR_LEVEL = 4, VWO_ERR_TOO_LARGE = 5, VWO_ERR_BOUNDARY = 6, VWO_ERR_ARG = 7
};

/* Wavelet identity codes for SymmetricAlignmentStrategy (identity checks). */
enum {
    VWO_WID_OTHER = 0, VWO_WID_HAAR = 1, VWO_WID_DB2 = 2, VWO_WID_DB4 = 4, VWO_WID_DB6 = 6,
    VWO_WID_DB8 = 8, VWO_WID_DB10 = 10, VWO_WID_SYM4 = 104, VWO_WID_SYM8 = 108,
    VWO_WID_COIF1 = 201, VWO_WID_COIF2 = 202, VWO_WID_COIF3 = 203, VWO_WID_COIF5 = 205
};

/* 1.0 / Math.sqrt(2.0): core/internal/ScalarOps.java:911, core/modwt/MODWTTransform.java:141 */
static double modwt_scale(void) { return 1.0 / sqrt(2.0); }

/* ---------------------------------------------------------------- A3 ---- */
/* MultiLevelMODWTTransform.calculateMaxLevels  core/modwt/MultiLevelMODWTTransform.java:455-501
 * (loop bound MAX_DECOMPOSITION_LEVELS = 10 at :117, so the result is <= 9). */
int vwo_max_levels(int signal_length, int filter_length)
{
    if (signal_length <= filter_length) return 0;
    int max_level = 1;
    long long lm1 = filter_length - 1;
    while (max_level < 10) {
        if (max_level - 1 >= 31) break;
        long long scaled = lm1 * (1LL << (max_level - 1)) + 1LL;
        if (scaled > signal_length) break;
        max_level++;
    }
    return max_level - 1;
}

/* Upsampled filter length L_j = (L-1)*2^(j-1)+1, ScalarOps.java:910-912 */
int vwo_upsampled_length(int L, int level)
{
    int up = (level <= 1) ? 1 : (1 << (level - 1));
    return (L - 1) * up + 1;
}

/* ---------------------------------------------------------------- A2 ---- */
/* ScalarOps.upsampleAndScaleForIMODWTSynthesis  core/internal/ScalarOps.java:909-916 */
int vwo_upsample_scale(const double *base, int L, int level, double *out)
{
    int up = (level <= 1) ? 1 : (1 << (level - 1));
    double scale = modwt_scale();
    int Lj = (L - 1) * up + 1;
    for (int i = 0; i < Lj; i++) out[i] = 0.0;
    for (int i = 0; i < L; i++) out[i * up] = base[i] * scale;
    return Lj;
}

/* QMF high-pass g[i] = (i even ? 1 : -1) * h[L-1-i]
 * core/api/Daubechies.java:323-330, core/api/Symlet.java:462-469, core/api/Coiflet.java:629-636 */
void vwo_qmf(const double *h, int L, double *g)
{
    for (int i = 0; i < L; i++) g[i] = (i % 2 == 0 ? 1 : -1) * h[L - 1 - i];
}

/* ------------------------------------------------------------- A7 mirror - */
/* MathUtils.symmetricBoundaryExtension  core/util/MathUtils.java:30-51 */
int vwo_symmetric_index(int idx, int n)
{
    if (idx >= 0 && idx < n) return idx;
    int period = 2 * n;
    idx = ((idx % period) + period) % period;
    if (idx >= n) idx = period - idx - 1;
    return idx;
}

/* Long rows: the per-output loops below run OpenMP-parallel over t (n >= 32768).  Each output is
 * still one sequential sum in the reference's order, so results are bit-identical to the serial
 * loops; inside an outer parallel region (batch over rows) they stay serial (no nesting). */

/* ---------------------------------------------------------------- A6 ---- */
/* ScalarOps.circularConvolveMODWTScalar  core/internal/ScalarOps.java:700-723 */
void vwo_circular_conv(const double *signal, int n, const double *filter, int fl, double *out)
{
    #pragma omp parallel for schedule(static) if (n >= 32768)
    for (int t = 0; t < n; t++) {
        double sum = 0.0;
        for (int l = 0; l < fl; l++) {
            int idx = t - l;
            int si;
            if (idx >= 0 && idx < n) si = idx;
            else if (idx < 0 && idx >= -n) si = idx + n;
            else si = ((idx % n) + n) % n;
            sum += signal[si] * filter[l];
        }
        out[t] = sum;
    }
}

/* MultiLevelMODWTTransform.circularConvolveMODWTDirect  core/modwt/MultiLevelMODWTTransform.java:763-787 */
void vwo_circular_conv_direct(const double *signal, int n, const double *filter, int fl, double *out)
{
    int eff = fl < n ? fl : n;
    #pragma omp parallel for schedule(static) if (n >= 32768)
    for (int t = 0; t < n; t++) {
        double sum = 0.0;
        int maxk = eff < t + 1 ? eff : t + 1;
        for (int k = 0; k < maxk; k++) sum += filter[k] * signal[t - k];
        for (int k = maxk; k < eff; k++) sum += filter[k] * signal[t - k + n];
        out[t] = sum;
    }
}

/* ScalarOps.zeroPaddingConvolveMODWT  core/internal/ScalarOps.java:790-808 */
void vwo_zero_conv(const double *signal, int n, const double *filter, int fl, double *out)
{
    #pragma omp parallel for schedule(static) if (n >= 32768)
    for (int t = 0; t < n; t++) {
        double sum = 0.0;
        for (int l = 0; l < fl; l++) {
            int si = t - l;
            if (si >= 0 && si < n) sum += signal[si] * filter[l];
        }
        out[t] = sum;
    }
}

/* ScalarOps.symmetricConvolveMODWT  core/internal/ScalarOps.java:818-835 */
void vwo_symmetric_conv(const double *signal, int n, const double *filter, int fl, double *out)
{
    #pragma omp parallel for schedule(static) if (n >= 32768)
    for (int t = 0; t < n; t++) {
        double sum = 0.0;
        for (int l = 0; l < fl; l++) {
            int idx = vwo_symmetric_index(t - l, n);
            sum += signal[idx] * filter[l];
        }
        out[t] = sum;
    }
}

/* ---------------------------------------------------------------- A8 ---- */
/* CoreFFT.fft, Cooley-Tukey default path  fft/CoreFFT.java:130-215 (no Stockham, no twiddle cache:
 * the twiddle recurrence below is the one the default path uses). */
static void core_fft(double *re, double *im, int n)
{
    if (n == 1) return;
    if (n == 2) {
        double r0 = re[0] + re[1], i0 = im[0] + im[1];
        double r1 = re[0] - re[1], i1 = im[0] - im[1];
        re[0] = r0; im[0] = i0; re[1] = r1; im[1] = i1;
        return;
    }
    int half = n / 2, j = half;
    for (int i = 1; i < n - 1; i++) {
        if (i < j) {
            double t = re[i]; re[i] = re[j]; re[j] = t;
            t = im[i]; im[i] = im[j]; im[j] = t;
        }
        int k = half;
        while (k <= j) { j -= k; k /= 2; }
        j += k;
    }
    for (int len = 2; len <= n; len *= 2) {
        double angle = -2 * M_PI / len;
        double wlr = cos(angle), wli = sin(angle);
        for (int i = 0; i < n; i += len) {
            double wr = 1.0, wi = 0.0;
            for (int j2 = 0; j2 < len / 2; j2++) {
                int u = i + j2, v = u + len / 2;
                double tr = re[v] * wr - im[v] * wi;
                double ti = re[v] * wi + im[v] * wr;
                re[v] = re[u] - tr;
                im[v] = im[u] - ti;
                re[u] += tr;
                im[u] += ti;
                double nwr = wr * wlr - wi * wli;
                double nwi = wr * wli + wi * wlr;
                wr = nwr; wi = nwi;
            }
        }
    }
}

/* CoreFFT.ifft  fft/CoreFFT.java:278-295 */
static void core_ifft(double *re, double *im, int n)
{
    for (int i = 0; i < n; i++) im[i] = -im[i];
    core_fft(re, im, n);
    for (int i = 0; i < n; i++) { re[i] /= n; im[i] = -im[i] / n; }
}

/* ScalarOps.circularConvolveMODWTFFT  core/internal/ScalarOps.java:650-681.
 * Zero-pads to nextPow2(N): circular only when N is a power of two. */
void vwo_fft_conv(const double *signal, int n, const double *filter, int fl, double *out)
{
    int m = 1;
    while (m < n) m <<= 1;
    double *xr = calloc(m, sizeof(double)), *xi = calloc(m, sizeof(double));
    double *hr = calloc(m, sizeof(double)), *hi = calloc(m, sizeof(double));
    memcpy(xr, signal, (size_t)n * sizeof(double));
    memcpy(hr, filter, (size_t)(fl < m ? fl : m) * sizeof(double));
    core_fft(xr, xi, m);
    core_fft(hr, hi, m);
    for (int k = 0; k < m; k++) {
        double r = xr[k] * hr[k] - xi[k] * hi[k];
        double im = xr[k] * hi[k] + xi[k] * hr[k];
        xr[k] = r; xi[k] = im;
    }
    core_ifft(xr, xi, m);
    for (int i = 0; i < n; i++) out[i] = xr[i];
    free(xr); free(xi); free(hr); free(hi);
}

/* FftHeuristics.shouldUseModwtFFT with defaults minN = 1024, ratio = 1/8
 * core/util/FftHeuristics.java:12-34 */
int vwo_should_use_fft(int n, int fl)
{
    if (n <= 0 || fl <= 0) return 0;
    if (n < 1024) return 0;
    return fl > n * (1.0 / 8.0);
}

/* WaveletOperations.circularConvolveMODWT  core/WaveletOperations.java:29-39 */
static void wavelet_ops_circular(const double *s, int n, const double *f, int fl, double *out)
{
    if (vwo_should_use_fft(n, fl)) vwo_fft_conv(s, n, f, fl, out);
    else vwo_circular_conv(s, n, f, fl, out);
}

/* -------------------------------------------------------------- A17 ----- */
/* ValidationUtils.validateFiniteValues  core/util/ValidationUtils.java:106-117 */
long long vwo_first_nonfinite(const double *v, long long n)
{
    for (long long i = 0; i < n; i++)
        if (!isfinite(v[i])) return i;
    return -1;
}

/* ------------------------------------------------------------ A4/A5 ----- */
/* MultiLevelMODWTTransform.applyScaledMODWT  core/modwt/MultiLevelMODWTTransform.java:710-757.
 * use_fft_switch = 1 reproduces the PERIODIC dispatch at :734-742 exactly. */
static int apply_scaled_modwt(const double *sig, int n, const double *lo, const double *hi, int fl,
                              int boundary, int use_fft_switch, double *approx, double *detail)
{
    if (fl > n) return VWO_ERR_TOO_LARGE;
    if (boundary == VWO_PERIODIC) {
        if (!use_fft_switch || n < 64 || fl > n / 2) {
            if (use_fft_switch) {
                vwo_circular_conv_direct(sig, n, lo, fl, approx);
                vwo_circular_conv_direct(sig, n, hi, fl, detail);
            } else {
                vwo_circular_conv(sig, n, lo, fl, approx);
                vwo_circular_conv(sig, n, hi, fl, detail);
            }
        } else {
            wavelet_ops_circular(sig, n, lo, fl, approx);
            wavelet_ops_circular(sig, n, hi, fl, detail);
        }
    } else if (boundary == VWO_ZERO_PADDING) {
        vwo_zero_conv(sig, n, lo, fl, approx);
        vwo_zero_conv(sig, n, hi, fl, detail);
    } else {
        vwo_symmetric_conv(sig, n, lo, fl, approx);
        vwo_symmetric_conv(sig, n, hi, fl, detail);
    }
    return VWO_OK;
}

/* MultiLevelMODWTTransform.decompose(signal, levels)  core/modwt/MultiLevelMODWTTransform.java:209-255.
 * details: [J][N] (level 1 first), approx: [N].  Returns a status code; *bad_index receives the
 * first non-finite index (A17).  check_levels=1 applies the core level cap (:225-239);
 * check_levels=0 gives BatchMODWT semantics (no cap, no validation, no FFT switch),
 * ext/extensions/modwt/BatchMODWT.java:90-111 + BatchSIMDMODWT.java:343-424 (whose per-lane
 * arithmetic -- `approxSum.add(samples.mul(scaledLow[l]))`, l ascending -- is K1's). */
int vwo_ml_decompose(const double *x, int n, const double *lo, const double *hi, int L,
                     int boundary, int levels, int core_semantics, double *details, double *approx,
                     long long *bad_index)
{
    if (bad_index) *bad_index = -1;
    if (!x || !lo || !hi) return VWO_ERR_NULL;
    if (core_semantics) {
        long long bad = vwo_first_nonfinite(x, n);
        if (bad >= 0) { if (bad_index) *bad_index = bad; return VWO_ERR_NONFINITE; }
    }
    if (n == 0) return VWO_ERR_EMPTY;
    if (boundary < 0 || boundary > 2) return VWO_ERR_BOUNDARY;
    if (core_semantics) {
        int maxl = vwo_max_levels(n, L);
        if (levels < 1 || levels > maxl) return VWO_ERR_LEVEL;
    } else if (levels < 1) {
        return VWO_ERR_LEVEL;
    }
    double *cur = malloc(sizeof(double) * n);
    double *nxt = malloc(sizeof(double) * n);
    int maxLj = vwo_upsampled_length(L, levels);
    double *flo = malloc(sizeof(double) * maxLj);
    double *fhi = malloc(sizeof(double) * maxLj);
    memcpy(cur, x, sizeof(double) * n);
    int st = VWO_OK;
    for (int level = 1; level <= levels; level++) {
        int fl = vwo_upsample_scale(lo, L, level, flo);
        vwo_upsample_scale(hi, L, level, fhi);
        if (core_semantics) {
            st = apply_scaled_modwt(cur, n, flo, fhi, fl, boundary, 1, nxt, details + (size_t)(level - 1) * n);
            if (st != VWO_OK) break;
            /* MODWTResult.create re-validates (core/modwt/MODWTResultImpl.java:47-48) */
            long long b1 = vwo_first_nonfinite(nxt, n), b2 = vwo_first_nonfinite(details + (size_t)(level - 1) * n, n);
            if (b1 >= 0 || b2 >= 0) { st = VWO_ERR_NONFINITE; if (bad_index) *bad_index = b1 >= 0 ? b1 : b2; break; }
        } else {
            /* BatchSIMDMODWT.generalBatchMODWTSoAWithScaledFilters :384-424 -- srcT = (t - l + N) % N */
            if (fl > n + 1) { st = VWO_ERR_TOO_LARGE; break; } /* Java would index out of bounds */
            double *d = details + (size_t)(level - 1) * n;
            #pragma omp parallel for schedule(static) if (n >= 32768)
            for (int t = 0; t < n; t++) {
                double as = 0.0, ds = 0.0;
                for (int l = 0; l < fl; l++) {
                    int src = (t - l + n) % n;
                    as = as + cur[src] * flo[l];
                    ds = ds + cur[src] * fhi[l];
                }
                nxt[t] = as; d[t] = ds;
            }
        }
        double *tmp = cur; cur = nxt; nxt = tmp;
    }
    if (st == VWO_OK) memcpy(approx, cur, sizeof(double) * n);
    free(cur); free(nxt); free(flo); free(fhi);
    return st;
}

/* --------------------------------------------------------------- A11 ---- */
/* SymmetricAlignmentStrategy.decide  core/modwt/SymmetricAlignmentStrategy.java:43-117.
 * The reference decides by object identity; wavelet_id carries that identity. */
void vwo_sym_decide(int wavelet_id, int L, int level, int *approx_plus, int *delta_h,
                    int *detail_plus, int *delta_g)
{
    int detailPlus = 1, deltaG, deltaH;
    int isHaar = (L <= 2);
    int approxPlus = isHaar;
    if (isHaar) {
        deltaG = 0;
        deltaH = (level <= 1) ? 0 : -1;
    } else {
        approxPlus = 0;
        if (wavelet_id == VWO_WID_DB6) {
            deltaH = (level <= 1) ? 0 : -1;
            deltaG = (level >= 3) ? 1 : 0;
        } else if (wavelet_id == VWO_WID_DB8) {
            deltaH = (level <= 1) ? 0 : 1;
            deltaG = (level >= 2) ? 1 : 0;
        } else if (wavelet_id == VWO_WID_SYM4) {
            approxPlus = 1; detailPlus = 0; deltaH = 0; deltaG = 0;
        } else if (wavelet_id == VWO_WID_SYM8) {
            approxPlus = 0;
            if (level <= 1) { deltaH = 0; deltaG = 0; }
            else if (level == 2) { deltaH = 1; deltaG = 0; }
            else { deltaH = 1; deltaG = 1; }
        } else if (wavelet_id == VWO_WID_COIF2) {
            approxPlus = 1; deltaH = (level <= 1) ? 0 : 1; detailPlus = 0; deltaG = 0;
        } else if (wavelet_id == VWO_WID_COIF3) {
            approxPlus = 0; detailPlus = 0;
            if (level <= 1) { deltaH = 0; deltaG = 0; } else { deltaH = -1; deltaG = 1; }
        } else if (L >= 12) {
            if (level <= 1) { deltaH = 0; deltaG = 0; }
            else { int even = (level % 2 == 0); deltaH = even ? 0 : -1; deltaG = even ? 0 : -1; }
        } else {
            if (level <= 1) { deltaH = 0; deltaG = 0; }
            else if (level == 2) { deltaH = -1; deltaG = 0; }
            else { deltaH = -1; deltaG = 0; }
        }
    }
    *approx_plus = approxPlus; *delta_h = deltaH; *detail_plus = detailPlus; *delta_g = deltaG;
}

/* MultiLevelMODWTTransform.computeTauJ  core/modwt/MultiLevelMODWTTransform.java:795-806 */
int vwo_compute_tau(int base_len, int level)
{
    int lm1 = base_len - 1;
    if (level <= 1) return lm1 / 2 > 0 ? lm1 / 2 : 0;
    long long up = 1LL << (level - 1);
    long long Lj = (long long)lm1 * up + 1LL;
    long long tau = (Lj - 1LL) / 2LL;
    if (tau < 0) return 0;
    if (tau > 2147483647LL) return 2147483647;
    return (int)tau;
}

/* MultiLevelMODWTTransform.applyScaledInverseMODWT  core/modwt/MultiLevelMODWTTransform.java:554-645 */
static int apply_scaled_inverse(const double *a, const double *d, int n, const double *lo, const double *hi,
                                int fl, int L, int wavelet_id, int boundary, int level, double *y)
{
    if (fl > n) return VWO_ERR_TOO_LARGE;
    if (boundary == VWO_PERIODIC) {
        #pragma omp parallel for schedule(static) if (n >= 32768)
        for (int t = 0; t < n; t++) {
            double sum = 0.0;
            for (int l = 0; l < fl; l++) sum += lo[l] * a[(t + l) % n];
            for (int l = 0; l < fl; l++) sum += hi[l] * d[(t + l) % n];
            y[t] = sum;
        }
    } else if (boundary == VWO_ZERO_PADDING) {
        #pragma omp parallel for schedule(static) if (n >= 32768)
        for (int t = 0; t < n; t++) {
            double sum = 0.0;
            for (int l = 0; l < fl; l++) {
                int idx = t + l;
                if (idx < n) sum += lo[l] * a[idx] + hi[l] * d[idx];
            }
            y[t] = sum;
        }
    } else {
        int ap, dh, dp, dg;
        vwo_sym_decide(wavelet_id, L, level, &ap, &dh, &dp, &dg);
        int tauH = vwo_compute_tau(L, level) + dh;
        int tauG = vwo_compute_tau(L, level) + dg;
        #pragma omp parallel for schedule(static) if (n >= 32768)
        for (int t = 0; t < n; t++) {
            double sum = 0.0;
            if (ap) { for (int l = 0; l < fl; l++) sum += lo[l] * a[vwo_symmetric_index(t + l - tauH, n)]; }
            else    { for (int l = 0; l < fl; l++) sum += lo[l] * a[vwo_symmetric_index(t - l + tauH, n)]; }
            if (dp) { for (int l = 0; l < fl; l++) sum += hi[l] * d[vwo_symmetric_index(t + l - tauG, n)]; }
            else    { for (int l = 0; l < fl; l++) sum += hi[l] * d[vwo_symmetric_index(t - l + tauG, n)]; }
            y[t] = sum;
        }
    }
    return VWO_OK;
}

/* MultiLevelMODWTTransform.reconstruct / reconstructFromLevel / reconstructLevels
 * core/modwt/MultiLevelMODWTTransform.java:339-349, :361-386, :398-446.
 * detail_mask bit (j-1) set = use d_j, clear = zero details at level j; approx_zero = start from
 * zeros (reconstructLevels with maxLevel < J).  details [J][N], approx [N]. */
int vwo_ml_reconstruct(const double *details, const double *approx, int n, const double *lo,
                       const double *hi, int L, int wavelet_id, int boundary, int levels,
                       unsigned detail_mask, int approx_zero, double *y)
{
    if (!details || !approx || !lo || !hi || !y) return VWO_ERR_NULL;
    if (n == 0) return VWO_ERR_EMPTY;
    if (boundary < 0 || boundary > 2) return VWO_ERR_BOUNDARY;
    if (levels < 1) return VWO_ERR_LEVEL;
    double *cur = malloc(sizeof(double) * n), *nxt = malloc(sizeof(double) * n);
    double *zero = calloc(n, sizeof(double));
    int maxLj = vwo_upsampled_length(L, levels);
    double *flo = malloc(sizeof(double) * maxLj), *fhi = malloc(sizeof(double) * maxLj);
    if (approx_zero) memset(cur, 0, sizeof(double) * n);
    else memcpy(cur, approx, sizeof(double) * n);
    int st = VWO_OK;
    for (int level = levels; level >= 1; level--) {
        int fl = vwo_upsample_scale(lo, L, level, flo);
        vwo_upsample_scale(hi, L, level, fhi);
        const double *d = ((detail_mask >> (level - 1)) & 1u) ? details + (size_t)(level - 1) * n : zero;
        st = apply_scaled_inverse(cur, d, n, flo, fhi, fl, L, wavelet_id, boundary, level, nxt);
        if (st != VWO_OK) break;
        double *t = cur; cur = nxt; nxt = t;
    }
    if (st == VWO_OK) memcpy(y, cur, sizeof(double) * n);
    free(cur); free(nxt); free(zero); free(flo); free(fhi);
    return st;
}

/* --------------------------------------------------------------- A12 ---- */
/* MODWTTransform.forward  core/modwt/MODWTTransform.java:131-189 (validation :369-414). */
int vwo_modwt_forward(const double *x, int n, const double *lo, const double *hi, int L,
                      int boundary, double *approx, double *detail, long long *bad_index)
{
    if (bad_index) *bad_index = -1;
    if (!x) return VWO_ERR_NULL;
    if (n == 0) return VWO_ERR_EMPTY;
    long long bad = vwo_first_nonfinite(x, n);
    if (bad >= 0) { if (bad_index) *bad_index = bad; return VWO_ERR_NONFINITE; }
    double s = modwt_scale();
    double *sl = malloc(sizeof(double) * L), *sh = malloc(sizeof(double) * L);
    for (int i = 0; i < L; i++) sl[i] = lo[i] * s;
    for (int i = 0; i < L; i++) sh[i] = hi[i] * s;
    if (boundary == VWO_PERIODIC) {
        wavelet_ops_circular(x, n, sl, L, approx);
        wavelet_ops_circular(x, n, sh, L, detail);
    } else if (boundary == VWO_ZERO_PADDING) {
        vwo_zero_conv(x, n, sl, L, approx);
        vwo_zero_conv(x, n, sh, L, detail);
    } else {
        vwo_symmetric_conv(x, n, sl, L, approx);
        vwo_symmetric_conv(x, n, sh, L, detail);
    }
    free(sl); free(sh);
    return VWO_OK;
}

/* MODWTTransform.inverse  core/modwt/MODWTTransform.java:203-299 (pairwise sums; SYMMETRIC t-l).
 * batch_optimized = 1 gives inverseBatchOptimized :619-689 (SYMMETRIC uses t+l). */
int vwo_modwt_inverse(const double *approx, const double *detail, int n, const double *lo,
                      const double *hi, int L, int boundary, int batch_optimized, double *y)
{
    if (!approx || !detail || !y) return VWO_ERR_NULL;
    if (n == 0) return VWO_ERR_EMPTY;
    double s = modwt_scale();
    double *sl = malloc(sizeof(double) * L), *sh = malloc(sizeof(double) * L);
    for (int i = 0; i < L; i++) sl[i] = lo[i] * s;
    for (int i = 0; i < L; i++) sh[i] = hi[i] * s;
    for (int t = 0; t < n; t++) {
        double sum = 0.0;
        for (int l = 0; l < L; l++) {
            int ci;
            if (boundary == VWO_PERIODIC) ci = (t + l) % n;
            else if (boundary == VWO_ZERO_PADDING) { ci = t + l; if (ci >= n) continue; }
            else if (!batch_optimized) ci = vwo_symmetric_index(t - l, n);
            else { int period = n << 1; int mod = (t + l) % period; ci = mod < n ? mod : period - mod - 1; }
            sum += sl[l] * approx[ci] + sh[l] * detail[ci];
        }
        y[t] = sum;
    }
    free(sl); free(sh);
    return VWO_OK;
}

/* ------------------------------------------------------------ A13-A15 --- */
/* VectorWaveSwtAdapter.decomposeSWT  core/swt/VectorWaveSwtAdapter.java:337-394 (never the FFT
 * branch); forwardParallel :210-290 computes the same numbers (convolvePeriodicChunk order is K1's). */
int vwo_swt_forward(const double *x, int n, const double *lo, const double *hi, int L, int boundary,
                    int levels, double *details, double *approx)
{
    int maxLj = vwo_upsampled_length(L, levels);
    double *flo = malloc(sizeof(double) * maxLj), *fhi = malloc(sizeof(double) * maxLj);
    double *cur = malloc(sizeof(double) * n), *nxt = malloc(sizeof(double) * n);
    memcpy(cur, x, sizeof(double) * n);
    for (int level = 1; level <= levels; level++) {
        int fl = vwo_upsample_scale(lo, L, level, flo);
        vwo_upsample_scale(hi, L, level, fhi);
        double *d = details + (size_t)(level - 1) * n;
        if (boundary == VWO_PERIODIC) { vwo_circular_conv(cur, n, flo, fl, nxt); vwo_circular_conv(cur, n, fhi, fl, d); }
        else if (boundary == VWO_ZERO_PADDING) { vwo_zero_conv(cur, n, flo, fl, nxt); vwo_zero_conv(cur, n, fhi, fl, d); }
        else { vwo_symmetric_conv(cur, n, flo, fl, nxt); vwo_symmetric_conv(cur, n, fhi, fl, d); }
        double *t = cur; cur = nxt; nxt = t;
    }
    memcpy(approx, cur, sizeof(double) * n);
    free(flo); free(fhi); free(cur); free(nxt);
    return VWO_OK;
}

/* VectorWaveSwtAdapter.reconstructPeriodic  core/swt/VectorWaveSwtAdapter.java:444-474 */
void vwo_swt_reconstruct_periodic(const double *details, const double *approx, int n, const double *lo,
                                  const double *hi, int L, int levels, double *y)
{
    int maxLj = vwo_upsampled_length(L, levels);
    double *h = malloc(sizeof(double) * maxLj), *g = malloc(sizeof(double) * maxLj);
    double *cur = malloc(sizeof(double) * n), *nxt = malloc(sizeof(double) * n);
    memcpy(cur, approx, sizeof(double) * n);
    for (int level = levels; level >= 1; level--) {
        const double *det = details + (size_t)(level - 1) * n;
        int Lh = vwo_upsample_scale(lo, L, level, h);
        int Lg = vwo_upsample_scale(hi, L, level, g);
        #pragma omp parallel for schedule(static) if (n >= 32768)
        for (int t = 0; t < n; t++) {
            double sum = 0.0;
            for (int l = 0; l < Lh; l++) sum += h[l] * cur[(t + l) % n];
            for (int l = 0; l < Lg; l++) sum += g[l] * det[(t + l) % n];
            nxt[t] = sum;
        }
        double *t = cur; cur = nxt; nxt = t;
    }
    memcpy(y, cur, sizeof(double) * n);
    free(h); free(g); free(cur); free(nxt);
}

/* Arrays.sort(double[]) order (Double.compare): NaN above +Inf, all NaNs equal.  The keys are |c|, so
 * the -0.0 < 0.0 rule never applies. */
static int cmp_double(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    if (isnan(x) || isnan(y)) return (isnan(x) != 0) - (isnan(y) != 0);
    return (x > y) - (x < y);
}

/* VectorWaveSwtAdapter.estimateNoiseSigma  core/swt/VectorWaveSwtAdapter.java:627-645 */
double vwo_noise_sigma(const double *coeffs, int n)
{
    double *a = malloc(sizeof(double) * n);
    for (int i = 0; i < n; i++) a[i] = fabs(coeffs[i]);
    qsort(a, n, sizeof(double), cmp_double);
    double median = (n % 2 == 0) ? (a[n / 2 - 1] + a[n / 2]) / 2.0 : a[n / 2];
    free(a);
    return median / 0.6745;
}

/* Universal threshold T = sigma * sqrt(2 * ln N)  core/swt/VectorWaveSwtAdapter.java:514 */
double vwo_universal_threshold(double sigma, int n) { return sigma * sqrt(2 * log((double)n)); }

/* MutableMultiLevelMODWTResult.applyThresholdToArray  core/modwt/MutableMultiLevelMODWTResult.java:97-114 */
void vwo_threshold(double *c, int n, double threshold, int soft)
{
    for (int i = 0; i < n; i++) {
        double av = fabs(c[i]);
        if (soft) {
            if (av > threshold) {
                double sg = c[i] > 0 ? 1.0 : (c[i] < 0 ? -1.0 : c[i]); /* Math.signum */
                c[i] = sg * (av - threshold);
            } else {
                c[i] = 0.0;
            }
        } else if (av <= threshold) {
            c[i] = 0.0;
        }
    }
}

/* VectorWaveSwtAdapter.denoise(signal, levels, threshold, soft)  core/swt/VectorWaveSwtAdapter.java:546-562
 * -> forward, applyUniversalThreshold (:505-520) or fixed threshold on all detail levels, inverse (:435-442).
 * sigma_out (optional) receives the MAD estimate (NaN if a fixed threshold was used). */
int vwo_swt_denoise(const double *x, int n, const double *lo, const double *hi, int L, int wavelet_id,
                    int boundary, int levels, double threshold, int soft, double *y, double *thr_out)
{
    double *det = malloc(sizeof(double) * (size_t)n * levels), *app = malloc(sizeof(double) * n);
    vwo_swt_forward(x, n, lo, hi, L, boundary, levels, det, app);
    double T = threshold;
    if (threshold < 0) {
        double sigma = vwo_noise_sigma(det, n);
        T = vwo_universal_threshold(sigma, n);
    }
    for (int level = 1; level <= levels; level++) vwo_threshold(det + (size_t)(level - 1) * n, n, T, soft);
    int st = VWO_OK;
    if (boundary == VWO_PERIODIC) vwo_swt_reconstruct_periodic(det, app, n, lo, hi, L, levels, y);
    else st = vwo_ml_reconstruct(det, app, n, lo, hi, L, wavelet_id, boundary, levels, 0xFFFFFFFFu, 0, y);
    if (thr_out) *thr_out = T;
    free(det); free(app);
    return st;
}

/* ------------------------------------------------------- WaveletDenoiser ---- */
/* core/denoising/WaveletDenoiser.java.  Methods: 0 UNIVERSAL, 1 SURE, 2 MINIMAX, 3 BAYES, 4 FIXED. */
enum { VWO_THR_UNIVERSAL = 0, VWO_THR_SURE = 1, VWO_THR_MINIMAX = 2, VWO_THR_BAYES = 3, VWO_THR_FIXED = 4 };

/* calculateSURERisk :477-492 -- sequential sum in coefficient order */
double vwo_sure_risk(const double *c, int n, double threshold, double sigma)
{
    double sigma2 = sigma * sigma;
    double risk = -n * sigma2;
    for (int i = 0; i < n; i++) {
        double absC = fabs(c[i]);
        if (absC <= threshold) risk += c[i] * c[i];
        else risk += sigma2 + (absC - threshold) * (absC - threshold);
    }
    return risk / n;
}

/* calculateSUREThreshold :441-472 -- every sorted |c| is tried (O(n^2)), first minimum kept, capped at
 * the universal threshold */
double vwo_sure_threshold(const double *c, int n, double sigma)
{
    double *s = malloc(sizeof(double) * (size_t)n);
    for (int i = 0; i < n; i++) s[i] = fabs(c[i]);
    qsort(s, n, sizeof(double), cmp_double);
    double minRisk = INFINITY, best = 0;
    for (int k = 0; k < n; k++) {
        double t = s[k];
        double risk = vwo_sure_risk(c, n, t, sigma);
        if (risk < minRisk) { minRisk = risk; best = t; }
    }
    free(s);
    double universal = sigma * sqrt(2.0 * log((double)n));
    if (best > universal) best = universal;
    return best;
}

/* calculateMinimaxThreshold :497-509 */
double vwo_minimax_threshold(int n, double sigma)
{
    double logN = log((double)n);
    if (n <= 32) return 0;
    if (n <= 64) return sigma * 0.3936 + 0.1829 * sigma * logN;
    return sigma * (0.4745 + 0.1148 * logN);
}

/* calculateBayesThreshold :521-549 -- sequential mean and variance, BAYES_EPSILON = 1e-10 (:62) */
double vwo_bayes_threshold(const double *c, int n, double sigma)
{
    double sigma2 = sigma * sigma;
    double mean = 0.0;
    for (int i = 0; i < n; i++) mean += c[i];
    mean /= n;
    double variance = 0.0;
    for (int i = 0; i < n; i++) {
        double diff = c[i] - mean;
        variance += diff * diff;
    }
    variance /= n;
    double sigmaX2 = variance - sigma2 > 0.0 ? variance - sigma2 : 0.0; /* Math.max(0.0, v - s2), finite */
    double sigmaX = sqrt(sigmaX2 + 1e-10);
    return sigma2 / sigmaX;
}

/* calculateThreshold :394-436 (FIXED -> error) */
int vwo_calc_threshold(const double *c, int n, double sigma, int method, double *out)
{
    switch (method) {
        case VWO_THR_UNIVERSAL: *out = sigma * sqrt(2.0 * log((double)n)); return VWO_OK;
        case VWO_THR_SURE: *out = vwo_sure_threshold(c, n, sigma); return VWO_OK;
        case VWO_THR_MINIMAX: *out = vwo_minimax_threshold(n, sigma); return VWO_OK;
        case VWO_THR_BAYES: *out = vwo_bayes_threshold(c, n, sigma); return VWO_OK;
        default: return VWO_ERR_ARG;
    }
}

/* denoise(signal, method, type) :124-143 (levels == 0; method FIXED = denoiseFixed :354-364 with
 * `fixed`), denoiseMultiLevel :155-170 with DenoisedMultiLevelResult's per-level thresholds :204-231
 * (sigma from d_1, level j uses sigma / Math.sqrt(1 << j) and its own coefficients).  thr_out holds
 * max(levels, 1) thresholds. */
int vwo_wavelet_denoise(const double *x, int n, const double *lo, const double *hi, int L, int wavelet_id,
                        int boundary, int levels, int method, double fixed, int soft, double *y, double *thr_out,
                        long long *bad_index)
{
    int st;
    if (levels == 0) {
        double *a = malloc(sizeof(double) * n), *d = malloc(sizeof(double) * n);
        st = vwo_modwt_forward(x, n, lo, hi, L, boundary, a, d, bad_index);
        double T = fixed;
        if (st == VWO_OK && method != VWO_THR_FIXED) st = vwo_calc_threshold(d, n, vwo_noise_sigma(d, n), method, &T);
        if (st == VWO_OK) {
            vwo_threshold(d, n, T, soft);
            vwo_modwt_inverse(a, d, n, lo, hi, L, boundary, 0, y);
            if (thr_out) thr_out[0] = T;
        }
        free(a); free(d);
        return st;
    }
    if (method == VWO_THR_FIXED) return VWO_ERR_ARG;
    double *det = malloc(sizeof(double) * (size_t)n * levels), *app = malloc(sizeof(double) * n);
    st = vwo_ml_decompose(x, n, lo, hi, L, boundary, levels, 1, det, app, bad_index);
    if (st == VWO_OK) {
        double sigma = vwo_noise_sigma(det, n);
        for (int level = 1; level <= levels && st == VWO_OK; level++) {
            double *dl = det + (size_t)(level - 1) * n;
            double levelScale = sqrt((double)(1 << level));
            double T = 0;
            st = vwo_calc_threshold(dl, n, sigma / levelScale, method, &T);
            vwo_threshold(dl, n, T, soft);
            if (thr_out) thr_out[level - 1] = T;
        }
    }
    if (st == VWO_OK) st = vwo_ml_reconstruct(det, app, n, lo, hi, L, wavelet_id, boundary, levels, 0xFFFFFFFFu, 0, y);
    free(det); free(app);
    return st;
}

/* --------------------------------------------------------------- A16 ---- */
/* BatchSIMDMODWT.batchMODWTSoA single level  ext/extensions/modwt/BatchSIMDMODWT.java:64-274.
 * Haar uses the hard-coded 0.5/-0.5 taps (:86-140); L == 4 takes the "db4" branch (:145-206). */
void vwo_batch_single(const double *x, int n, const double *lo, const double *hi, int L, int is_haar,
                      double *approx, double *detail)
{
    double s = modwt_scale();
    if (is_haar) {
        for (int t = 0; t < n; t++) {
            int tm1 = (t - 1 + n) % n;
            approx[t] = x[t] * 0.5 + x[tm1] * 0.5;
            detail[t] = x[t] * 0.5 + x[tm1] * -0.5;
        }
        return;
    }
    double sl[64], sh[64];
    for (int i = 0; i < L; i++) { sl[i] = lo[i] * s; sh[i] = hi[i] * s; }
    for (int t = 0; t < n; t++) {
        double as = 0.0, ds = 0.0;
        for (int l = 0; l < L; l++) {
            int src = (t - l + n) % n;
            as = as + x[src] * sl[l];
            ds = ds + x[src] * sh[l];
        }
        approx[t] = as; detail[t] = ds;
    }
}

/* BatchSIMDMODWT.generalBatchMODWTSoAWithScaledFiltersAndHistory  ext/extensions/modwt/BatchSIMDMODWT.java:447-507
 * One signal: history [hist_len] (oldest first), block [n]. */
void vwo_conv_with_history(const double *hist, int hist_len, const double *x, int n, const double *flo,
                           const double *fhi, int fl, double *approx, double *detail)
{
    for (int t = 0; t < n; t++) {
        double as = 0.0, ds = 0.0;
        for (int l = 0; l < fl; l++) {
            int idx = t - l;
            double v = idx >= 0 ? x[idx] : hist[hist_len + idx];
            as = as + v * flo[l];
            ds = ds + v * fhi[l];
        }
        approx[t] = as; detail[t] = ds;
    }
}

/* ------------------------------------------------- CPU baseline (bench) - */
/* Batched core decompose + reconstruct (PERIODIC, core semantics), OpenMP over signals.
 * This is the "scalar-core CPU path" the north star times beside the GPU: exactly the Java loops,
 * zero taps included.  Returns the number of threads used. */
int vwo_batch_fwd_inv(const double *x, long long B, int n, const double *lo, const double *hi, int L,
                      int wavelet_id, int boundary, int levels, double *y)
{
    int threads = 1;
#ifdef _OPENMP
    threads = omp_get_max_threads();
#endif
    #pragma omp parallel
    {
        double *det = malloc(sizeof(double) * (size_t)n * levels);
        double *app = malloc(sizeof(double) * n);
        #pragma omp for schedule(dynamic, 1)
        for (long long b = 0; b < B; b++) {
            vwo_ml_decompose(x + (size_t)b * n, n, lo, hi, L, boundary, levels, 1, det, app, NULL);
            vwo_ml_reconstruct(det, app, n, lo, hi, L, wavelet_id, boundary, levels, 0xFFFFFFFFu, 0,
                               y + (size_t)b * n);
        }
        free(det); free(app);
    }
    return threads;
}

/* Batched SWT denoise (config 3 CPU baseline). */
int vwo_batch_denoise(const double *x, long long B, int n, const double *lo, const double *hi, int L,
                      int wavelet_id, int boundary, int levels, double threshold, int soft, double *y)
{
    int threads = 1;
#ifdef _OPENMP
    threads = omp_get_max_threads();
#endif
    #pragma omp parallel for schedule(dynamic, 1)
    for (long long b = 0; b < B; b++)
        vwo_swt_denoise(x + (size_t)b * n, n, lo, hi, L, wavelet_id, boundary, levels, threshold, soft,
                        y + (size_t)b * n, NULL);
    return threads;
}

/* Counter-based synthetic input, SURVEY.md §8(d): u = (splitmix64(seed ^ (b*N+i)) >> 11) * 2^-53, x = 2u - 1.
 * The engine's device generator (vw_fill_uniform) produces the same bits. */
static uint64_t splitmix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void vwo_fill_uniform(double *x, long long count, unsigned long long seed, long long offset)
{
    for (long long i = 0; i < count; i++) {
        uint64_t r = splitmix64((uint64_t)seed ^ (uint64_t)(offset + i));
        double u = (double)(r >> 11) * (1.0 / 9007199254740992.0);
        x[i] = 2.0 * u - 1.0;
    }
}
