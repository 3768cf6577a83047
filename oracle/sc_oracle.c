/*
 * sc_oracle.c -- CPU restatement of the SurfCascade detect path
 * (TEST INFRASTRUCTURE ONLY -- see sc_oracle.h for the rules and the parity
 * status).  Scalar C; every f32/f64 operation is written in the association
 * order the reference's SSE code imposes.  Build with -ffp-contract=off and
 * without -ffast-math (oracle/Makefile) so each C operator is one IEEE op.
 */
#include "sc_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ----------------------------------------------------------------------- */
/* Scan geometry                                                            */
/* ----------------------------------------------------------------------- */

/* l = (int)(70 * pow(1.1, i)) in f64 -- ObjDetector.cpp:180. */
int sco_level_len(int base, int i) { return (int)(base * pow(1.1, i)); }

/* (int)min(log(W/(float)70)/log(1.1), log(H/(float)70)/log(1.1)) + 1 levels
 * (the loop at ObjDetector.cpp:178 is inclusive).  log() of a float argument
 * resolves to the float overload in MSVC C++ (ObjDetector.cpp:174). */
int sco_num_levels(int W, int H, int base_w, int base_h) {
    double a = logf((float)W / (float)base_w) / log(1.1);
    double b = logf((float)H / (float)base_h) / log(1.1);
    return (int)(a < b ? a : b) + 1;
}

/* step = win.width > 20 ? win.width / 20 : 1 -- ObjDetector.cpp:139. */
int sco_step(const sco_params *p) {
    if (p->step > 0) return p->step;
    return p->base_len > 20 ? p->base_len / 20 : 1;
}

int sco_effective_levels(int W, int H, const sco_params *p) {
    if (p->n_levels >= 0) return p->n_levels;
    return sco_num_levels(W, H, p->base_len, p->base_len * p->aspect_h);
}

int64_t sco_grid_count(int W, int H, const sco_params *p) {
    int st = sco_step(p), nl = sco_effective_levels(W, H, p);
    int64_t n = 0;
    for (int i = 0; i < nl; i++) {
        int l = sco_level_len(p->base_len, i), lh = l * p->aspect_h;
        if (l > W || lh > H) continue;
        n += (int64_t)((W - l) / st + 1) * ((H - lh) / st + 1);
    }
    return n;
}

/* Dense template patches -- DenseSURFFeatureExtractor.cpp:21,49-63 and
 * constants .h:31-35: shapes {2x2, 1x4, 4x1}, cell edge 6..W/2, stride 4. */
int sco_extract_patches(int tw, int th, int32_t *rects, int cap) {
    static const int shp[3][2] = {{2, 2}, {1, 4}, {4, 1}};
    int n = 0;
    for (int j = 0; j < 3; j++)
        for (int c = 6; c <= tw / 2; c++) {
            int pw = shp[j][0] * c, ph = shp[j][1] * c;
            for (int y = 0; y + ph <= th; y += 4)
                for (int x = 0; x + pw <= tw; x += 4) {
                    if (rects && n < cap) {
                        rects[4 * n + 0] = x;
                        rects[4 * n + 1] = y;
                        rects[4 * n + 2] = pw;
                        rects[4 * n + 3] = ph;
                    }
                    n++;
                }
        }
    return n;
}

/* ----------------------------------------------------------------------- */
/* Gradient planes + integral table                                         */
/* ----------------------------------------------------------------------- */

static inline uint8_t sat_sub(int a, int b) { return (uint8_t)(a > b ? a - b : 0); }

/* T2bFilter -- DenseSURFFeatureExtractor.cpp:199-349.  For each direction k
 * the pair (Ip, In) gives plane 2k = sat(Ip - In) = (|d|-d)/2 and plane
 * 2k+1 = sat(In - Ip) = (|d|+d)/2 with d = In - Ip.  Edge handling of the
 * reference reduces to clamping the neighbour coordinates:
 *   dx (:224-254)  In = I[y][x+1]      Ip = I[y][x-1]
 *   dy (:256-281)  In = I[y+1][x]      Ip = I[y-1][x]
 *   du (:283-314)  In = I[y+1][x+1]    Ip = I[y-1][x-1]
 *   dv (:316-347)  In = I[y-1][x+1]    Ip = I[y+1][x-1]
 * (W, H >= 2). */
void sco_gradients(const uint8_t *img, int W, int H, int stride, uint8_t *g) {
    const size_t sz = (size_t)W * H;
    for (int y = 0; y < H; y++) {
        const uint8_t *c = img + (size_t)y * stride;
        const uint8_t *u = img + (size_t)(y > 0 ? y - 1 : 0) * stride;
        const uint8_t *d = img + (size_t)(y < H - 1 ? y + 1 : H - 1) * stride;
        for (int x = 0; x < W; x++) {
            int xn = x < W - 1 ? x + 1 : W - 1, xp = x > 0 ? x - 1 : 0;
            size_t o = (size_t)y * W + x;
            int in, ip;
            in = c[xn]; ip = c[xp];
            g[0 * sz + o] = sat_sub(ip, in); g[1 * sz + o] = sat_sub(in, ip);
            in = d[x]; ip = u[x];
            g[2 * sz + o] = sat_sub(ip, in); g[3 * sz + o] = sat_sub(in, ip);
            in = d[xn]; ip = u[xp];
            g[4 * sz + o] = sat_sub(ip, in); g[5 * sz + o] = sat_sub(in, ip);
            in = u[xn]; ip = d[xp];
            g[6 * sz + o] = sat_sub(ip, in); g[7 * sz + o] = sat_sub(in, ip);
        }
    }
}

/* IntegralImage -- DenseSURFFeatureExtractor.cpp:65-87: cv::integral
 * (8U -> 32F) per plane, then cv::merge into the 8-float-per-cell table
 * (F256Dat, .h:21-25).  OpenCV's scalar integral_ keeps the running row sum
 * s in the sum type (f32, exact here since s <= 255*W < 2^24) and forms
 * S[y+1][x+1] = S[y][x+1] + s as one f32 add, sequential in y.
 * T has (H+1) rows of (W+1) cells of 8 floats. */
void sco_integral(const uint8_t *img, int W, int H, int stride, float *T) {
    const size_t sz = (size_t)W * H, pitch = (size_t)(W + 1) * 8;
    uint8_t *g = (uint8_t *)malloc(8 * sz);
    sco_gradients(img, W, H, stride, g);
    memset(T, 0, pitch * sizeof(float));
    for (int y = 0; y < H; y++) {
        float *prev = T + (size_t)y * pitch, *row = T + (size_t)(y + 1) * pitch;
        for (int ch = 0; ch < 8; ch++) {
            const uint8_t *gr = g + ch * sz + (size_t)y * W;
            float s = 0.0f;
            row[ch] = 0.0f;
            for (int x = 0; x < W; x++) {
                s += (float)gr[x];
                row[(size_t)(x + 1) * 8 + ch] = prev[(size_t)(x + 1) * 8 + ch] + s;
            }
        }
    }
    free(g);
}

/* ----------------------------------------------------------------------- */
/* Window arithmetic                                                        */
/* ----------------------------------------------------------------------- */

#define CELL(T, W, yy, xx) ((T) + ((size_t)(yy) * (size_t)((W) + 1) + (size_t)(xx)) * 8)

/* sum(win) -- DenseSURFFeatureExtractor.cpp:351-358 (xmm_f1 = channels 0-3,
 * (A+D)-(B+C) per lane, then ((s0+s1)+s2)+s3, /2), compared at
 * ObjDetector.cpp:188 against win.area()*6 converted to float. */
int sco_prefilter(const float *T, int W, int x, int y, int w, int h, float k,
                  float *m_out) {
    const float *tl = CELL(T, W, y, x), *br = CELL(T, W, y + h, x + w);
    const float *tr = CELL(T, W, y, x + w), *bl = CELL(T, W, y + h, x);
    float v[4];
    for (int c = 0; c < 4; c++) v[c] = (tl[c] + br[c]) - (tr[c] + bl[c]);
    float m = (((v[0] + v[1]) + v[2]) + v[3]) / 2.0f;
    if (m_out) *m_out = m;
    float thr = (float)(w * h) * k;
    return m > thr;
}

/* ProjectPatches -- DenseSURFFeatureExtractor.cpp:459-484.  scale is
 * (float)l / tmpl_w (f32 division); coordinates truncate toward zero. */
void sco_project(const int32_t tr[4], float scale, int wx, int wy,
                 int32_t out[4]) {
    out[0] = (int)((float)tr[0] * scale) + wx;
    out[1] = (int)((float)tr[1] * scale) + wy;
    if (tr[2] >= tr[3]) {
        int ratio = tr[2] / tr[3];
        out[3] = (int)((float)tr[3] * scale);
        out[2] = out[3] * ratio;
    } else {
        int ratio = tr[3] / tr[2];
        out[2] = (int)((float)tr[2] * scale);
        out[3] = out[2] * ratio;
    }
}

/* SSE3 hadd-ordered sum of squares with lane-3 seed FLT_EPSILON --
 * DenseSURFFeatureExtractor.cpp:427-433: c_k = (q0+q1)+(q2+q3) per quad,
 * SS = (((eps + c0) + c1) + ...) + c7. */
static float ss_hadd(const float f[32]) {
    float ss = FLT_EPSILON;
    for (int k = 0; k < 8; k++) {
        float q0 = f[4 * k] * f[4 * k], q1 = f[4 * k + 1] * f[4 * k + 1];
        float q2 = f[4 * k + 2] * f[4 * k + 2], q3 = f[4 * k + 3] * f[4 * k + 3];
        float ck = (q0 + q1) + (q2 + q3);
        ss = ss + ck;
    }
    return ss;
}

/* Normalize -- DenseSURFFeatureExtractor.cpp:417-457; theta = 2/sqrt(32)
 * (.h:36).  _mm_min_ps(a,b) = a<b?a:b and _mm_max_ps(a,b) = a>b?a:b. */
void sco_normalize(float f[32]) {
    const float theta = 2.0f / sqrtf(32.0f);
    float t = sqrtf(ss_hadd(f)) * theta, nt = -t;
    for (int i = 0; i < 32; i++) {
        float v = f[i] < t ? f[i] : t;
        f[i] = v > nt ? v : nt;
    }
    float r = 1.0f / sqrtf(ss_hadd(f));
    for (int i = 0; i < 32; i++) f[i] = f[i] * r;
}

/* GetRectsFromPatch (:360-377) + CalcFeature (:379-415): four cells,
 * feature[8*cell + ch] = (TL + BR) - (TR + BL), then Normalize. */
void sco_calc_feature(const float *T, int W, const int32_t r[4], float f[32]) {
    int ce = (r[2] == r[3]) ? r[2] / 2 : (r[2] < r[3] ? r[2] : r[3]);
    int gw = r[2] / ce, gh = r[3] / ce;
    for (int hh = 0; hh < gh; hh++)
        for (int ww = 0; ww < gw; ww++) {
            int cell = hh * gw + ww;
            int x0 = r[0] + ww * ce, y0 = r[1] + hh * ce;
            const float *tl = CELL(T, W, y0, x0), *br = CELL(T, W, y0 + ce, x0 + ce);
            const float *tr = CELL(T, W, y0, x0 + ce), *bl = CELL(T, W, y0 + ce, x0);
            for (int c = 0; c < 8; c++)
                f[8 * cell + c] = (tl[c] + br[c]) - (tr[c] + bl[c]);
        }
    sco_normalize(f);
}

/* LogisticRegression::Predict -- LogisticRegression.cpp:46-68: four f32
 * lane accumulators over i = 0,4,..,28, two hadds, then f64:
 * z += w[32]*bias, p = 1/(1+exp(-z)), returned as float. */
float sco_lr_predict(const float *w, double bias, const float f[32]) {
    float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int i = 0; i < 32; i += 4)
        for (int j = 0; j < 4; j++) s[j] = w[i + j] * f[i + j] + s[j];
    float z32 = (s[0] + s[1]) + (s[2] + s[3]);
    double prob = (double)z32;
    prob += (double)w[32] * bias;
    prob = 1.0 / (1.0 + exp(-prob));
    return (float)prob;
}

/* GentleAdaboost::Predict2 -- GentleAdaboost.cpp:247-261: f32 sum in weak
 * order, divided by (float)n. */
static float stage_score(const float *T, int W, const sco_model *m, int s,
                         int64_t off, float scale, int x, int y) {
    float sum = 0.0f;
    for (int k = 0; k < m->n_weak[s]; k++) {
        int32_t pr[4];
        float f[32];
        sco_project(m->patch + 4 * (off + k), scale, x, y, pr);
        sco_calc_feature(T, W, pr, f);
        sum += sco_lr_predict(m->w + 33 * (off + k), m->bias[off + k], f);
    }
    return sum / (float)m->n_weak[s];
}

/* One window of the detect loop, ObjDetector.cpp:188-201: prefilter, then
 * stages until the first stage whose score < theta.  Returns p (the failing
 * stage, n_stages if all pass, -1 if the prefilter rejects); *s_last gets the
 * last evaluated stage score. */
int sco_eval_window(const float *T, int W, const sco_model *m, int l, int lh,
                    int x, int y, float k, float *s_last, float *stage_scores) {
    if (!sco_prefilter(T, W, x, y, l, lh, k, NULL)) return -1;
    float scale = (float)l / (float)m->tmpl_w;
    int p;
    float score = 0.0f;
    int64_t off = 0;
    for (p = 0; p < m->n_stages; p++) {
        score = stage_score(T, W, m, p, off, scale, x, y);
        if (stage_scores) stage_scores[p] = score;
        off += m->n_weak[p];
        if ((double)score < (double)m->theta[p]) break;
    }
    if (s_last) *s_last = score;
    return p;
}

/* Every stage score of a window, no early exit (threshold calibration). */
void sco_all_stage_scores(const float *T, int W, const sco_model *m, int l,
                          int x, int y, float *out) {
    float scale = (float)l / (float)m->tmpl_w;
    int64_t off = 0;
    for (int s = 0; s < m->n_stages; s++) {
        out[s] = stage_score(T, W, m, s, off, scale, x, y);
        off += m->n_weak[s];
    }
}

/* Score of one stage for a batch of windows (l[i], x[i], y[i]); used to
 * calibrate the synthetic models' thetas (tests/golden/make_models.py). */
void sco_stage_score_batch(const float *T, int W, const sco_model *m,
                           const int32_t *l, const int32_t *x, const int32_t *y,
                           int64_t n, int stage, float *out, int nthreads) {
    int64_t off = 0;
    for (int s = 0; s < stage; s++) off += m->n_weak[s];
    (void)nthreads;
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
    for (int64_t i = 0; i < n; i++) {
        float scale = (float)l[i] / (float)m->tmpl_w;
        out[i] = stage_score(T, W, m, stage, off, scale, x[i], y[i]);
    }
}

/* final = (score + p + 1) / S in f64 -- ObjDetector.cpp:201. */
static double final_score(float s_last, int p, int S) {
    return ((double)s_last + p + 1) / S;
}

/* Every window of the stride-step grid (all levels), canonical order
 * (level, y, x): p_out = stage reached (-1 = prefilter reject), s_out = last
 * stage score (0 for prefilter rejects). */
int64_t sco_eval_grid(const float *T, int W, int H, const sco_model *m,
                      const sco_params *p, int16_t *p_out, float *s_out,
                      int nthreads) {
    int st = sco_step(p), nl = sco_effective_levels(W, H, p);
    int64_t *base = (int64_t *)calloc((size_t)nl + 1, sizeof(int64_t));
    for (int i = 0; i < nl; i++) {
        int l = sco_level_len(p->base_len, i), lh = l * p->aspect_h;
        int64_t n = (l > W || lh > H) ? 0 : (int64_t)((W - l) / st + 1) * ((H - lh) / st + 1);
        base[i + 1] = base[i] + n;
    }
    int64_t total = base[nl];
    (void)nthreads;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for (int i = 0; i < nl; i++) {
        int l = sco_level_len(p->base_len, i), lh = l * p->aspect_h;
        if (l > W || lh > H) continue;
        int nx = (W - l) / st + 1;
        int64_t o = base[i];
        for (int y = 0; y <= H - lh; y += st)
            for (int xi = 0; xi < nx; xi++, o++) {
                float s = 0.0f;
                int pr = sco_eval_window(T, W, m, l, lh, xi * st, y, p->prefilter_k, &s, NULL);
                p_out[o] = (int16_t)pr;
                s_out[o] = pr < 0 ? 0.0f : s;
            }
    }
    free(base);
    return total;
}

static int cmp_window(const void *a, const void *b) {
    const sco_window *u = (const sco_window *)a, *v = (const sco_window *)b;
    if (u->level != v->level) return u->level < v->level ? -1 : 1;
    if (u->y != v->y) return u->y < v->y ? -1 : 1;
    if (u->x != v->x) return u->x < v->x ? -1 : 1;
    return 0;
}

/* The reference detect loop, ObjDetector.cpp:174-220: OpenMP over levels
 * (static schedule, :177), rows at stride `step`, the serial x chain with
 * the adaptive stride multi (:185-186, :214-217), detections collected under
 * a critical section (:203-212).  Output is sorted canonically by
 * (level, y, x) because the reference's append order is nondeterministic.
 * Returns the number of detections (may exceed cap; only cap are stored). */
int64_t sco_detect(const float *T, int W, int H, const sco_model *m,
                   const sco_params *p, sco_window *out, int64_t cap,
                   int64_t *n_visited, int nthreads) {
    int st = sco_step(p), nl = sco_effective_levels(W, H, p);
    const int S = m->n_stages;
    int64_t n_det = 0, visited = 0;
    int64_t buf_cap = 1024;
    sco_window *buf = (sco_window *)malloc(sizeof(sco_window) * buf_cap);
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : visited)
    for (int i = 0; i < nl; i++) {
        int l = sco_level_len(p->base_len, i), lh = l * p->aspect_h;
        for (int y = 0; y <= H - lh; y += st) {
            int multi = 1;
            for (int x = 0; x <= W - l; x += multi * st) {
                visited++;
                float s = 0.0f;
                int pr = sco_eval_window(T, W, m, l, lh, x, y, p->prefilter_k, &s, NULL);
                if (pr < 0) {
                    multi = 2;
                    continue;
                }
                double score = final_score(s, pr, S);
                if (pr == S) {
#pragma omp critical(sco_collect)
                    {
                        if (n_det == buf_cap) {
                            buf_cap *= 2;
                            buf = (sco_window *)realloc(buf, sizeof(sco_window) * buf_cap);
                        }
                        sco_window wv = {i, x, y, l, lh, pr, score};
                        buf[n_det++] = wv;
                    }
                }
                multi = (score < p->stride_score) ? 2 : 1;
            }
        }
    }
    qsort(buf, (size_t)n_det, sizeof(sco_window), cmp_window);
    if (out) memcpy(out, buf, sizeof(sco_window) * (size_t)(n_det < cap ? n_det : cap));
    free(buf);
    if (n_visited) *n_visited = visited;
    return n_det;
}

/* The adaptive-stride x walk (ObjDetector.cpp:185-217) over per-window
 * results already computed for the whole stride-`step` grid (sco_eval_grid's
 * output, canonical level / row / x order): visited[g] = 1 for every window
 * the reference's loop visits.  The same recurrence as sco_detect: after a
 * prefilter reject or a final score < stride_score the chain skips a window.
 * layout: per level (nx, ny, grid base).  Returns the visited count. */
int64_t sco_walk_grid(const int16_t *p_grid, const float *s_grid, const int64_t *layout,
                      int n_levels, int n_stages, double stride_score, uint8_t *visited) {
    int64_t nv = 0;
    for (int i = 0; i < n_levels; i++) {
        const int64_t nx = layout[3 * i], ny = layout[3 * i + 1], base = layout[3 * i + 2];
        for (int64_t r = 0; r < ny; r++) {
            const int64_t o = base + r * nx;
            for (int64_t j = 0; j < nx;) {
                visited[o + j] = 1;
                nv++;
                const int pr = p_grid[o + j];
                if (pr < 0) {
                    j += 2;
                    continue;
                }
                j += final_score(s_grid[o + j], pr, n_stages) < stride_score ? 2 : 1;
            }
        }
    }
    return nv;
}

/* ---- exposure to the unpinned third-party arithmetic -------
 * Over the windows the reference visits (the sco_detect loop), counts:
 *  st[0] weak evaluations; st[1] / st[2] those whose f64 sigmoid
 *  1/(1+exp(-z)) (LogisticRegression.cpp:65) lies within 2 / 16 ulp(f64) of
 *  an f32 rounding boundary -- where a CRT exp() 1-2 ulp away from glibc's
 *  could change the (float) cast;
 *  st[3] stage decisions (ObjDetector.cpp:197), st[4] those with the stage
 *  score within one f32 ulp of theta;
 *  st[5] windows with a final score (prefilter passed), st[6] those whose
 *  final score (s + p + 1)/S lies within one f32 ulp of 0.5 (:214).
 *  st[7] integral sums above 2^24 among the table's channel values (the
 *  order-sensitive regime of cv::integral: an IPP route adding in another
 *  order could differ there). */
static int near_f32_boundary(double y, int ulps) {
    float f = (float)y;
    double lo = (double)nextafterf(f, -INFINITY), hi = (double)nextafterf(f, INFINITY);
    double m1 = ((double)f + hi) * 0.5, m2 = ((double)f + lo) * 0.5;  /* exact in f64 */
    double u = nextafter(y, INFINITY) - y;
    double d = fmin(fabs(y - m1), fabs(y - m2));
    return d <= ulps * u;
}

void sco_exposure(const float *T, int W, int H, const sco_model *m, const sco_params *p,
                  int64_t st[8], int nthreads) {
    int stp = sco_step(p), nl = sco_effective_levels(W, H, p);
    const int S = m->n_stages;
    int64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;
#pragma omp parallel for schedule(dynamic) num_threads(nthreads > 0 ? nthreads : 1) \
    reduction(+ : a0, a1, a2, a3, a4, a5, a6)
    for (int i = 0; i < nl; i++) {
        int l = sco_level_len(p->base_len, i), lh = l * p->aspect_h;
        float scale = (float)l / (float)m->tmpl_w;
        for (int y = 0; y <= H - lh; y += stp) {
            int multi = 1;
            for (int x = 0; x <= W - l; x += multi * stp) {
                if (!sco_prefilter(T, W, x, y, l, lh, p->prefilter_k, NULL)) {
                    multi = 2;
                    continue;
                }
                int pr;
                float score = 0.0f;
                int64_t off = 0;
                for (pr = 0; pr < S; pr++) {
                    float sum = 0.0f;
                    for (int k = 0; k < m->n_weak[pr]; k++) {
                        const float *w = m->w + 33 * (off + k);
                        int32_t rc[4];
                        float f[32];
                        sco_project(m->patch + 4 * (off + k), scale, x, y, rc);
                        sco_calc_feature(T, W, rc, f);
                        float s4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                        for (int q = 0; q < 32; q += 4)
                            for (int j = 0; j < 4; j++) s4[j] = w[q + j] * f[q + j] + s4[j];
                        double z = (double)((s4[0] + s4[1]) + (s4[2] + s4[3]));
                        z += (double)w[32] * m->bias[off + k];
                        double yv = 1.0 / (1.0 + exp(-z));
                        a0++;
                        a1 += near_f32_boundary(yv, 2);
                        a2 += near_f32_boundary(yv, 16);
                        sum += (float)yv;
                    }
                    score = sum / (float)m->n_weak[pr];
                    off += m->n_weak[pr];
                    a3++;
                    float th = m->theta[pr];
                    a4 += fabsf(score - th) <= nextafterf(th, INFINITY) - th;
                    if ((double)score < (double)th) break;
                }
                double fin = final_score(score, pr, S);
                a5++;
                a6 += fabs(fin - p->stride_score) <= (double)(nextafterf(0.5f, INFINITY) - 0.5f);
                multi = fin < p->stride_score ? 2 : 1;
            }
        }
    }
    for (int64_t c = 0; c < (int64_t)(W + 1) * (H + 1) * 8; c++) a7 += T[c] > 16777216.0f;
    st[0] = a0; st[1] = a1; st[2] = a2; st[3] = a3; st[4] = a4; st[5] = a5; st[6] = a6; st[7] = a7;
}

/* ---- exp() sensitivity, exact (VERDICT r2 Next 6) ----------
 * The reference's sigmoid calls the MSVC CRT exp (LogisticRegression.cpp:65),
 * which is not in /root/reference.  Model: the CRT result e' lies within one
 * f64 ulp of glibc's e = exp(-z) (both are faithful; glibc's is correctly
 * rounded on these arguments, checked with mpmath by profiles/exposure.py).
 * Over the windows the reference visits (the sco_detect chain), every weak
 * evaluation is recomputed with e' = nextafter(e, -inf) and nextafter(e, +inf)
 * through the reference's f64 ops, 1.0/(1.0 + e'), cast to float.  A weak
 * "flips" when such an alternative f32 differs from the baseline.  For every
 * flipping alternative the window is re-evaluated with that one weak output
 * replaced, and when the window's result (p, s_last) changes, the row's x
 * chain is re-walked from it until it rejoins the baseline chain; detections
 * that appear or vanish on the way are counted.
 *  st[0] weak evaluations             st[1] evaluations with a flipping alternative
 *  st[2] flipping alternatives        st[3] alternatives that flip a stage decision
 *  st[4] alternatives that change the window's (p, s_last) bits
 *  st[5] alternatives that change the window's stride (good / skip)
 *  st[6] detections that appear or vanish (window itself + chain re-walk)
 *  st[7] windows with two or more flipping evaluations
 *  st[8] alternatives that leave a detection a detection with other score
 *        bits (a 1-ulp change of s_last: ~1e-8 on (s + S + 1)/S, inside
 *        north_star's 1e-5 score tolerance)
 * zd: the z of the first zcap flipping evaluations (for the mpmath check). */
static float lr_alt(const float *w, double bias, const float f[32], float *alt_lo, float *alt_hi,
                    double *z_out) {
    float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int i = 0; i < 32; i += 4)
        for (int j = 0; j < 4; j++) s[j] = w[i + j] * f[i + j] + s[j];
    float z32 = (s[0] + s[1]) + (s[2] + s[3]);
    double z = (double)z32;
    z += (double)w[32] * bias;
    double e = exp(-z);
    *z_out = z;
    *alt_lo = (float)(1.0 / (1.0 + nextafter(e, -INFINITY)));
    *alt_hi = (float)(1.0 / (1.0 + nextafter(e, INFINITY)));
    return (float)(1.0 / (1.0 + e));
}

/* sco_eval_window with weak g's output replaced by v (g < 0: none). */
static int eval_window_ovr(const float *T, int W, const sco_model *m, int l, int lh, int x, int y,
                           float k, float *s_last, int64_t g, float v) {
    if (!sco_prefilter(T, W, x, y, l, lh, k, NULL)) return -1;
    float scale = (float)l / (float)m->tmpl_w;
    int p;
    float score = 0.0f;
    int64_t off = 0;
    for (p = 0; p < m->n_stages; p++) {
        float sum = 0.0f;
        for (int q = 0; q < m->n_weak[p]; q++) {
            if (off + q == g) {
                sum += v;
                continue;
            }
            int32_t pr[4];
            float f[32];
            sco_project(m->patch + 4 * (off + q), scale, x, y, pr);
            sco_calc_feature(T, W, pr, f);
            sum += sco_lr_predict(m->w + 33 * (off + q), m->bias[off + q], f);
        }
        score = sum / (float)m->n_weak[p];
        off += m->n_weak[p];
        if ((double)score < (double)m->theta[p]) break;
    }
    *s_last = score;
    return p;
}

void sco_exp_sensitivity(const float *T, int W, int H, const sco_model *m, const sco_params *p,
                         int64_t st[9], double *zd, int64_t zcap, int nthreads) {
    int stp = sco_step(p), nl = sco_effective_levels(W, H, p);
    const int S = m->n_stages;
    int64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0, a8 = 0, nz = 0;
#pragma omp parallel for schedule(dynamic) num_threads(nthreads > 0 ? nthreads : 1) \
    reduction(+ : a0, a1, a2, a3, a4, a5, a6, a7, a8)
    for (int i = 0; i < nl; i++) {
        int l = sco_level_len(p->base_len, i), lh = l * p->aspect_h;
        if (l > W || lh > H) continue;
        int nx = (W - l) / stp + 1;
        float scale = (float)l / (float)m->tmpl_w;
        /* per row: baseline results of the visited windows (-3: not visited) */
        int *bp = (int *)malloc(sizeof(int) * nx);
        float *bs = (float *)malloc(sizeof(float) * nx);
        /* flips of the row: (window, weak, alternative value) */
        int64_t fcap = 64, nf = 0;
        int64_t *fw = (int64_t *)malloc(sizeof(int64_t) * 2 * fcap);
        float *fv = (float *)malloc(sizeof(float) * fcap);
        for (int y = 0; y <= H - lh; y += stp) {
            for (int j = 0; j < nx; j++) bp[j] = -3;
            nf = 0;
            int multi = 1;
            for (int j = 0; j < nx; j += multi) {
                int x = j * stp;
                if (!sco_prefilter(T, W, x, y, l, lh, p->prefilter_k, NULL)) {
                    bp[j] = -1;
                    bs[j] = 0.0f;
                    multi = 2;
                    continue;
                }
                int pr, nflip = 0;
                float score = 0.0f;
                int64_t off = 0;
                for (pr = 0; pr < S; pr++) {
                    float sum = 0.0f;
                    for (int q = 0; q < m->n_weak[pr]; q++) {
                        int32_t rc[4];
                        float f[32], lo, hi;
                        double z;
                        sco_project(m->patch + 4 * (off + q), scale, x, y, rc);
                        sco_calc_feature(T, W, rc, f);
                        float v = lr_alt(m->w + 33 * (off + q), m->bias[off + q], f, &lo, &hi, &z);
                        a0++;
                        if (lo != v || hi != v) {
                            a1++;
                            nflip++;
#pragma omp critical(sco_zd)
                            {
                                if (zd && nz < zcap) zd[nz] = z;
                                nz++;
                            }
                            float alts[2] = {lo, hi};
                            for (int u = 0; u < 2; u++) {
                                if (alts[u] == v || (u == 1 && alts[1] == alts[0])) continue;
                                if (nf == fcap) {
                                    fcap *= 2;
                                    fw = (int64_t *)realloc(fw, sizeof(int64_t) * 2 * fcap);
                                    fv = (float *)realloc(fv, sizeof(float) * fcap);
                                }
                                fw[2 * nf] = j;
                                fw[2 * nf + 1] = off + q;
                                fv[nf++] = alts[u];
                            }
                        }
                        sum += v;
                    }
                    score = sum / (float)m->n_weak[pr];
                    off += m->n_weak[pr];
                    if ((double)score < (double)m->theta[pr]) break;
                }
                a7 += nflip >= 2;
                bp[j] = pr;
                bs[j] = score;
                multi = final_score(score, pr, S) < p->stride_score ? 2 : 1;
            }
            /* every flipping alternative of the row, one at a time */
            for (int64_t t = 0; t < nf; t++) {
                const int j = (int)fw[2 * t];
                const int64_t g = fw[2 * t + 1];
                a2++;
                float s2;
                int p2 = eval_window_ovr(T, W, m, l, lh, j * stp, y, p->prefilter_k, &s2, g, fv[t]);
                if (p2 == bp[j] && s2 == bs[j]) continue;
                a4++;
                /* the stage decision that flipped: the first stage where they part */
                a3 += p2 != bp[j];
                const int good0 = !(final_score(bs[j], bp[j], S) < p->stride_score);
                const int good2 = !(final_score(s2, p2, S) < p->stride_score);
                const int det0 = bp[j] == S, det2 = p2 == S;
                a6 += det0 != det2;
                a8 += det0 && det2 && s2 != bs[j];
                if (good0 == good2) continue;
                a5++;
                /* re-walk the chain from j with the alternative until it lands
                 * on a window the baseline chain visits (identical after that) */
                int k2 = j + (good2 ? 1 : 2);
                int kb = j + (good0 ? 1 : 2);  /* baseline chain's next visit */
                while (k2 < nx) {
                    while (kb < k2 && kb < nx) {  /* baseline windows skipped by the new chain */
                        if (bp[kb] == S) a6++;
                        kb += (bp[kb] < 0 || final_score(bs[kb], bp[kb], S) < p->stride_score) ? 2 : 1;
                    }
                    if (kb == k2) break;  /* rejoined */
                    float s3;
                    int p3 = eval_window_ovr(T, W, m, l, lh, k2 * stp, y, p->prefilter_k, &s3, -1, 0.0f);
                    if (p3 == S) a6++;    /* a window only the new chain visits */
                    k2 += (p3 < 0 || final_score(s3, p3, S) < p->stride_score) ? 2 : 1;
                }
                while (k2 >= nx && kb < nx) {  /* the new chain left the row first */
                    if (bp[kb] == S) a6++;
                    kb += (bp[kb] < 0 || final_score(bs[kb], bp[kb], S) < p->stride_score) ? 2 : 1;
                }
            }
        }
        free(bp);
        free(bs);
        free(fw);
        free(fv);
    }
    st[0] = a0; st[1] = a1; st[2] = a2; st[3] = a3; st[4] = a4; st[5] = a5; st[6] = a6; st[7] = a7;
    st[8] = a8;
}

/* In-memory u8 frame -> raw detections (the reference's per-image body,
 * ObjDetector.cpp:165-220, without decode / file I/O). */
int64_t sco_detect_frame(const uint8_t *img, int W, int H, int stride,
                         const sco_model *m, const sco_params *p,
                         sco_window *out, int64_t cap, int64_t *n_visited,
                         int nthreads, float *scratch_T) {
    float *T = scratch_T;
    if (!T) T = (float *)malloc(sizeof(float) * (size_t)(W + 1) * (H + 1) * 8);
    sco_integral(img, W, H, stride, T);
    int64_t n = sco_detect(T, W, H, m, p, out, cap, n_visited, nthreads);
    if (!scratch_T) free(T);
    return n;
}

/* Hard-negative scan of one image -- DenseSURFFeatureExtractor::FillNegSamples
 * (DenseSURFFeatureExtractor.cpp:124-195): levels l_k = (int)(tw * 1.1^k),
 * k = 0..(int)min(log(W/(float)tw)/log(1.1), log(H/(float)tw)/log(1.1))
 * (:146, :153; the height term also divides by size.width), square l x l
 * windows with rows and columns at stride 10 (:155, :161), no prefilter.  A
 * window is a candidate when the cascade accepts it (CascadeClassifier::
 * Predict, CascadeClassifier.cpp:63-72: no stage's GentleAdaboost::Predict is
 * below its theta) -- with no stage yet ("first", :170) every window is.
 * Candidates in (level, y, x) order; the first `cap` get their ExtractFeatures
 * descriptors (:88-93) over all n_patches template patches, ProjectPatches'd
 * to the window: feat[(i*n_patches + j)*32 + c].  The reference appends them
 * from OpenMP threads in a nondeterministic order and stops at n_total; the
 * candidate set is what is deterministic.  Returns the candidate count. */
int64_t sco_mine(const float *T, int W, int H, const sco_model *m, const int32_t *patches,
                 int n_patches, sco_window *out, float *feat, int64_t cap, int nthreads) {
    const int tw = m->tmpl_w, nl = sco_num_levels(W, H, tw, tw);
    if (nl <= 0) return 0;
    sco_window **lv = (sco_window **)calloc((size_t)nl, sizeof(sco_window *));
    int64_t *cnt = (int64_t *)calloc((size_t)nl, sizeof(int64_t));
    int i;
#pragma omp parallel for schedule(dynamic) num_threads(nthreads > 0 ? nthreads : 1)
    for (i = 0; i < nl; i++) {
        int l = sco_level_len(tw, i);
        if (l > W || l > H) continue;
        int64_t n = 0, c = (int64_t)((H - l) / 10 + 1) * ((W - l) / 10 + 1);
        lv[i] = (sco_window *)malloc(sizeof(sco_window) * (size_t)c);
        for (int y = 0; y <= H - l; y += 10)
            for (int x = 0; x + l <= W; x += 10) {
                float s_last = 0.0f;
                int p = sco_eval_window(T, W, m, l, l, x, y, -INFINITY, &s_last, NULL);
                if (p == m->n_stages) {
                    sco_window wv = {i, x, y, l, l, p, (double)s_last};
                    lv[i][n++] = wv;
                }
            }
        cnt[i] = n;
    }
    int64_t total = 0;
    for (i = 0; i < nl; i++) {
        for (int64_t k = 0; k < cnt[i]; k++) {
            if (total < cap) {
                sco_window wv = lv[i][k];
                if (out) out[total] = wv;
                if (feat) {
                    float scale = (float)wv.w / (float)tw;
                    for (int j = 0; j < n_patches; j++) {
                        int32_t pr[4];
                        sco_project(patches + 4 * j, scale, wv.x, wv.y, pr);
                        sco_calc_feature(T, W, pr, feat + ((size_t)total * n_patches + j) * 32);
                    }
                }
            }
            total++;
        }
        free(lv[i]);
    }
    free(lv);
    free(cnt);
    return total;
}
