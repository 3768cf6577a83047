#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "sc_oracle.h"
/* early-exit analysis: items needed when a stage's decision is taken as soon
   as the f32 partial-sum bounds decide it (checks every `chunk` weaks) */
static double fin(float s, int p, int S) { return ((double)s + p + 1) / S; }
void ee_stats(const float *T, int W, int H, const sco_model *m, const sco_params *pp, int nchunk,
              const int *chunks, int64_t *out /* [2 + nchunk] */) {
    int st = sco_step(pp), nl = sco_effective_levels(W, H, pp);
    const int S = m->n_stages;
    int maxn = 0; for (int s = 0; s < S; s++) if (m->n_weak[s] > maxn) maxn = m->n_weak[s];
    float *pr = malloc(sizeof(float) * maxn);
    for (int i = 0; i < nl; i++) {
        int l = sco_level_len(pp->base_len, i), lh = l * pp->aspect_h;
        float scale = (float)l / (float)m->tmpl_w;
        for (int y = 0; y <= H - lh; y += st) {
            int multi = 1;
            for (int x = 0; x <= W - l; x += multi * st) {
                if (!sco_prefilter(T, W, x, y, l, lh, pp->prefilter_k, NULL)) { multi = 2; continue; }
                int64_t off = 0; int p; float score = 0;
                for (p = 0; p < S; p++) {
                    int n = m->n_weak[p];
                    float sum = 0;
                    for (int k = 0; k < n; k++) {
                        int32_t r[4]; float f[32];
                        sco_project(m->patch + 4 * (off + k), scale, x, y, r);
                        sco_calc_feature(T, W, r, f);
                        pr[k] = sco_lr_predict(m->w + 33 * (off + k), m->bias[off + k], f);
                    }
                    out[0] += n;
                    /* decided-at k for every k */
                    int kstar = n;
                    float Sk = 0;
                    for (int k = 0; k <= n; k++) {
                        if (k > 0) Sk += pr[k - 1];
                        if (k == n) break;
                        float U = Sk; for (int j = k; j < n; j++) U += 1.0f;
                        float sl = Sk / (float)n, su = U / (float)n;
                        if ((double)su < (double)m->theta[p]) {
                            if ((fin(sl, p, S) < pp->stride_score) == (fin(su, p, S) < pp->stride_score)) { kstar = k; break; }
                        } else if (p < S - 1 && (double)sl >= (double)m->theta[p]) { kstar = k; break; }
                    }
                    out[1] += kstar;
                    for (int c = 0; c < nchunk; c++) {
                        int ch = chunks[c];
                        int kc = ((kstar + ch - 1) / ch) * ch; if (kc > n) kc = n;
                        out[2 + c] += kc;
                    }
                    for (int k = 0; k < n; k++) sum += pr[k];
                    score = sum / (float)n;
                    off += n;
                    if ((double)score < (double)m->theta[p]) break;
                }
                multi = fin(score, p, S) < pp->stride_score ? 2 : 1;
            }
        }
    }
    free(pr);
}
