/* l2sim.c -- trace-driven model of the chain kernel's L1 / L2 traffic
 * (profiling tool; VERDICT r2 Next 1: find why the wide levels miss L2).
 *
 * Input (from l2sim.py): per XCD, the chain kernel's tasks in queue order;
 * per task, its evaluated windows and, stage by stage, the (survivor, weak)
 * items in the kernel's k-major order.  The model:
 *   - XCD x runs `conc` tasks at once (32 CUs x waves x 2 slots), dealt to
 *     its CUs round-robin; the active tasks advance in turn, one item
 *     iteration (64 items) at a time, a finished task replaced by the next
 *     one in the queue (the chain kernel's dequeue);
 *   - an item iteration is 20 wave-level loads (10 corner slots x 2 channel
 *     halves); each load's 64 lanes touch a set of 128-B lines, each distinct
 *     line one L1 access (TCP tag lookups are 64-B sectors on gfx950, lines
 *     are 128 B: profiles/calib);
 *   - L1: 32 KiB per CU = 256 lines of 128 B, 16-way LRU;
 *   - L2: 4 MiB per XCD, 128-B lines, 16-way, 2048 sets, LRU; set index
 *     hashed from the line address (XOR fold).
 * Not modelled: the prefilter's loads, timing (hand-off waits, rounds of
 * unequal length), the Infinity Cache behind L2.
 * Output: per level group, L1 accesses / misses and L2 hits / misses. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int ways, sets;
    uint64_t *tag;  /* [sets][ways], 0 = empty (tags stored +1) */
    uint32_t *age;  /* LRU stamps */
    uint32_t clock;
} Cache;

static void cache_init(Cache *c, int lines, int ways) {
    c->ways = ways;
    c->sets = lines / ways;
    c->tag = calloc((size_t)lines, sizeof(uint64_t));
    c->age = calloc((size_t)lines, sizeof(uint32_t));
    c->clock = 0;
}
static void cache_free(Cache *c) {
    free(c->tag);
    free(c->age);
}
static inline uint32_t set_of(const Cache *c, uint64_t line) {
    uint64_t h = line ^ (line >> 11) ^ (line >> 22);
    return (uint32_t)(h % (uint64_t)c->sets);
}
/* returns 1 on hit; inserts on miss */
static inline int cache_access(Cache *c, uint64_t line) {
    const uint32_t s = set_of(c, line);
    uint64_t *t = c->tag + (size_t)s * c->ways;
    uint32_t *a = c->age + (size_t)s * c->ways;
    const uint64_t key = line + 1;
    int victim = 0;
    uint32_t oldest = UINT32_MAX;
    c->clock++;
    for (int w = 0; w < c->ways; w++) {
        if (t[w] == key) {
            a[w] = c->clock;
            return 1;
        }
        if (t[w] == 0) {
            victim = w;
            oldest = 0;
        } else if (a[w] < oldest) {
            oldest = a[w];
            victim = w;
        }
    }
    t[victim] = key;
    a[victim] = c->clock;
    return 0;
}

typedef struct {
    int W, H, step, ph, Qp, rowp, hs, cs; /* table geometry (sc_kernels.hpp TableGeom) */
} Geom;

static inline int64_t cell_of(const Geom *g, int y, int x, int h) {
    return (int64_t)y * g->rowp + (int64_t)g->cs * ((x % g->ph) * g->Qp + x / g->ph) + (int64_t)h * g->hs;
}

/* Per item: the 20 float4 cells (10 slots x 2 halves) of its patch's corners
 * (CalcFeature's uniform 10-slot set, sc_device.hpp corner_offsets). */
static void item_cells(const Geom *g, const int32_t *rect, float scale, int y, int x, int64_t out[20]) {
    const int px = (int)((float)rect[0] * scale), py = (int)((float)rect[1] * scale);
    const int e = (int)((float)rect[2] * scale), shape = rect[3];
    const int c = shape == 0 ? e / 2 : e;
    int ro[5], co[5];
    for (int i = 0; i < 5; i++) {
        ro[i] = y + py + i * c;
        co[i] = x + px + i * c;
    }
    for (int m = 0; m < 10; m++) {
        int r, cc;
        if (shape == 0) {
            r = m < 9 ? m / 3 : 2;
            cc = m < 9 ? m % 3 : 2;
        } else if (shape == 1) {
            r = m / 2;
            cc = m % 2;
        } else {
            r = m / 5;
            cc = m % 5;
        }
        out[m] = cell_of(g, ro[r], co[cc], 0);
        out[10 + m] = cell_of(g, ro[r], co[cc], 1);
    }
}

/* tasks: [n_tasks] offsets into items (items of task t: it_off[t] .. it_off[t+1]);
 * items: (level, y, j, k) int32 x 4; rects [K][4]; scale, l [levels];
 * xcd_of_task [n_tasks]; grp_of_level [levels]; stats out [n_groups][4]:
 * L1 accesses, L1 misses, L2 hits, L2 misses. */
/* big_slots >= 0: two queues per XCD -- slots s < big_slots take the earliest
 * task of either class (the class of a task = grp_of_level of its level, 1 =
 * big), the other slots only class-0 tasks (concurrency limit for the wide
 * levels); big_slots < 0: one queue. */
static int g_cell_bytes = 16; /* 12: u24-packed half cells (lossless for values < 2^24) */
void l2sim_set_cell_bytes(int b) { g_cell_bytes = b; }
/* cu_chunk > 0: a CU takes cu_chunk consecutive queue tasks at a time into
 * its own sub-queue (an LDS queue per workgroup), its slots then take tasks
 * from it: the tasks in flight on one CU are neighbouring rows */
static int g_cu_chunk = 0;
void l2sim_set_cu_chunk(int c) { g_cu_chunk = c; }
/* pair = 1: two lanes per item, lane h loading channel half h, so one wave
 * load covers corner slot m of 32 items in both halves (10 loads per
 * iteration of 32 items instead of 20 per 64); meant with the interleaved
 * 32-B cell layout, where an item's two halves share a line */
static int g_pair = 0;
void l2sim_set_pair(int p) { g_pair = p; }
int l2sim_run(const Geom *g, int n_tasks, const int64_t *it_off, const int32_t *items,
              const int32_t *rects, const float *scale, int conc, int cus, int l1_lines,
              int l2_lines, const int32_t *xcd_of_task, const int32_t *grp_of_level, int n_groups,
              int64_t *stats, int big_slots, const int32_t *grp_of_weak, const int32_t *alt_of_weak,
              const Geom *g2, int64_t alt_base) {
    memset(stats, 0, sizeof(int64_t) * 4 * n_groups);
    for (int x = 0; x < 8; x++) {
        /* this XCD's tasks in queue order */
        int nt = 0;
        for (int t = 0; t < n_tasks; t++) nt += xcd_of_task[t] == x;
        if (nt == 0) continue;
        int *q = malloc(sizeof(int) * nt);
        nt = 0;
        for (int t = 0; t < n_tasks; t++)
            if (xcd_of_task[t] == x) q[nt++] = t;
        Cache l2;
        cache_init(&l2, l2_lines, 16);
        Cache *l1 = malloc(sizeof(Cache) * cus);
        for (int c = 0; c < cus; c++) cache_init(&l1[c], l1_lines, 16);
        int *act = malloc(sizeof(int) * conc);     /* active task per slot (-1 idle) */
        int64_t *pos = malloc(sizeof(int64_t) * conc);
        /* class-split queues (big_slots >= 0): qs = small tasks, qb = big */
        int *qs = malloc(sizeof(int) * nt), *qb = malloc(sizeof(int) * nt);
        int ns = 0, nb = 0, is = 0, ib = 0;
        for (int i = 0; i < nt; i++) {
            if (big_slots >= 0 && grp_of_level[items[4 * it_off[q[i]]]] == 1) qb[nb++] = q[i];
            else qs[ns++] = q[i];
        }
        int next = 0, live = 0;
        const int chunk = g_cu_chunk > 0 ? g_cu_chunk : 1;
        int *cq = malloc(sizeof(int) * cus * chunk), *cqn = calloc(cus, sizeof(int)), *cqi = calloc(cus, sizeof(int));
        /* next task for slot s (-1: none) */
#define TAKE_CU(cu_) \
        (cqi[cu_] < cqn[cu_] ? cq[(cu_) * chunk + cqi[cu_]++] \
         : (cqn[cu_] = 0, cqi[cu_] = 0, ({ while (cqn[cu_] < chunk && next < nt) cq[(cu_) * chunk + cqn[cu_]++] = q[next++]; 0; }), \
            cqi[cu_] < cqn[cu_] ? cq[(cu_) * chunk + cqi[cu_]++] : -1))
#define TAKE(s_)                                                                        \
        ((big_slots < 0) ? (g_cu_chunk > 0 ? TAKE_CU((s_) % cus) : (next < nt ? q[next++] : -1)) \
         : ((s_) < big_slots                                                             \
                ? ((is < ns && (ib >= nb || qs[is] < qb[ib])) ? qs[is++] : (ib < nb ? qb[ib++] : -1)) \
                : (is < ns ? qs[is++] : -1)))
        for (int s = 0; s < conc; s++) {
            act[s] = TAKE(s);
            pos[s] = act[s] >= 0 ? it_off[act[s]] : 0;
            live += act[s] >= 0;
        }
        int64_t cells[64][20];
        uint64_t lines[128];
        while (live > 0) {
            for (int s = 0; s < conc; s++) {
                int t = act[s];
                if (t < 0) continue;
                const int64_t end = it_off[t + 1];
                const int per = g_pair ? 32 : 64;
                const int n = (int)((end - pos[s]) < per ? (end - pos[s]) : per);
                const int cu = s % cus;
                int grp = 0;
                for (int i = 0; i < n; i++) {
                    const int32_t *it = items + 4 * (pos[s] + i);
                    grp = grp_of_weak ? grp_of_weak[it[3]] : grp_of_level[it[0]];
                    if (alt_of_weak && alt_of_weak[it[3]]) {
                        item_cells(g2, rects + 4 * it[3], scale[it[0]], it[1], g->step * it[2], cells[i]);
                        for (int m = 0; m < 20; m++) cells[i][m] += alt_base;
                    } else {
                        item_cells(g, rects + 4 * it[3], scale[it[0]], it[1], g->step * it[2], cells[i]);
                    }
                }
                /* 20 wave-level loads (10 in pair mode); distinct lines per load = L1 accesses */
                for (int m = 0; m < (g_pair ? 10 : 20); m++) {
                    int nl = 0;
                    for (int i = 0; i < 2 * n * (g_pair ? 2 : 1); i++) {
                        /* pair: entries (item, half, first/last byte); else (item, first/last byte) */
                        const int it_i = g_pair ? i >> 2 : i >> 1, mm = g_pair ? m + 10 * ((i >> 1) & 1) : m;
                        const uint64_t b0 = (uint64_t)(cells[it_i][mm] * g_cell_bytes);
                        const uint64_t ln = (i & 1) ? (b0 + g_cell_bytes - 1) >> 7 : b0 >> 7;
                        int seen = 0;
                        for (int u = 0; u < nl; u++)
                            if (lines[u] == ln) {
                                seen = 1;
                                break;
                            }
                        if (!seen) lines[nl++] = ln;
                    }
                    int64_t *st = stats + 4 * grp;
                    for (int u = 0; u < nl; u++) {
                        st[0]++;
                        if (!cache_access(&l1[cu], lines[u])) {
                            st[1]++;
                            if (cache_access(&l2, lines[u])) st[2]++;
                            else st[3]++;
                        }
                    }
                }
                pos[s] += n;
                if (pos[s] >= end) {
                    act[s] = TAKE(s);
                    if (act[s] >= 0) pos[s] = it_off[act[s]];
                    else live--;
                }
            }
        }
        free(cq);
        free(cqn);
        free(cqi);
        free(qs);
        free(qb);
        free(act);
        free(pos);
        for (int c = 0; c < cus; c++) cache_free(&l1[c]);
        free(l1);
        cache_free(&l2);
        free(q);
    }
    return 0;
}
