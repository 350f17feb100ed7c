/*
 * graph_sparse.c — CPU restatement of MaskClustering's graph stages S2–S6 for
 * ScanNet++ / Matterport-sized scenes.  TEST
 * INFRASTRUCTURE ONLY: the checker the HIP path is compared against at sizes
 * where mcgraph_oracle.c's dense matrices (P×F point-in-mask, N×M contained
 * rows, N×N adjacency: 3 GB / 6.4 GB / 6.4 GB at C3) do not fit a test.  It is
 * never linked into, loaded by or called from the product library.
 *
 * Same semantics as mcgraph_oracle.c, which the golden fixtures pin to the
 * reference itself (tests/golden/make_golden.py); the CPU suite also pins this
 * file to those fixtures (tests/test_oracle_golden.py).  The data structures
 * differ: sparse rows instead of dense matrices, and the supporter counts by
 * column expansion instead of a dense C·Cᵀ.
 *
 *   S2  build_point_in_mask_matrix   graph/construction.py:22-64
 *   S3  process_one_mask / masks     graph/construction.py:98-170
 *   S4  get_observer_num_thresholds  graph/construction.py:80-96 (histogram; thresholds
 *                                    by orc_thresholds of mcgraph_oracle.c)
 *   S6  update_graph / cluster_into_new_nodes / iterative_clustering
 *                                    graph/iterative_clustering.py:5-43, graph/node.py:24-37
 *
 * Float semantics as mcgraph_oracle.c: S3 ratios in double, the S6 rate and
 * thresholds in float32 (volatile temporaries, built with -ffp-contract=off).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

static int cmp_i64(const void *a, const void *b)
{
    int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return x < y ? -1 : x > y;
}

/* ------------------------------------------------------------------------ */
/* S2 (construction.py:46-62).  Masks in frame order, ids ascending per frame.
 * kept[g] = 0 for the masks of a frame whose union is empty (:50-51).
 * boundary[p] = 1 if p lies in >= 2 masks of one frame (:56,62).
 * Per point list (pt_off[P+1], pt_ent[]) of the kept masks g holding it, ascending g
 * (frames ascending), for the S3 walk.  Returns the number of kept masks. */
int orcs_s2(int64_t P, int F, int M_in, const int32_t *col, const int64_t *off, const int32_t *pts,
            uint8_t *kept, uint8_t *boundary, int64_t *pt_off, int32_t *pt_ent)
{
    (void)F;
    int M = 0;
    for (int g = 0; g < M_in;) {
        int g1 = g;
        int64_t npts = 0;
        while (g1 < M_in && col[g1] == col[g]) { npts += off[g1 + 1] - off[g1]; g1++; }
        for (int h = g; h < g1; h++) { kept[h] = npts > 0; M += npts > 0; }
        g = g1;
    }
    memset(boundary, 0, (size_t)P);
    memset(pt_off, 0, (size_t)(P + 1) * sizeof(int64_t));
    for (int g = 0; g < M_in; g++)
        if (kept[g])
            for (int64_t k = off[g]; k < off[g + 1]; k++) pt_off[pts[k] + 1]++;
    for (int64_t p = 0; p < P; p++) pt_off[p + 1] += pt_off[p];
    int64_t *fill = (int64_t *)malloc((size_t)(P + 1) * sizeof(int64_t));
    memcpy(fill, pt_off, (size_t)(P + 1) * sizeof(int64_t));
    for (int g = 0; g < M_in; g++)   /* ascending g: every point's list is ascending */
        if (kept[g])
            for (int64_t k = off[g]; k < off[g + 1]; k++) pt_ent[fill[pts[k]]++] = g;
    free(fill);
    /* a point twice in one frame is a boundary point (frames ascending in the list) */
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < P; p++)
        for (int64_t k = pt_off[p] + 1; k < pt_off[p + 1]; k++)
            if (col[pt_ent[k]] == col[pt_ent[k - 1]]) boundary[p] = 1;
    return M;
}

/* ------------------------------------------------------------------------ */
/* S3 (construction.py:98-135) for every kept mask, then the under-segmentation undo
 * (:160-169).  Input g indexes the input masks; gidx[g] = global index of a kept mask,
 * -1 otherwise.  Output per global mask row r: up to F (frame, target) entries with the
 * contained global mask of each frame, ascending frames, after the undo (VF row = their
 * frames), as ct_len[r] entries at ct[r * F_cap ...].  useg[r] = under-segmented.
 * Returns |U|. */
int orcs_s3(int M_in, const int32_t *col, const int32_t *label, const int64_t *off, const int32_t *pts,
            const uint8_t *kept, const int32_t *gidx, const uint8_t *boundary, const int64_t *pt_off,
            const int32_t *pt_ent, double mask_visible_threshold, double contained_threshold,
            double undersegment_filter_threshold, int F_cap, int32_t *ct_frame, int32_t *ct_tgt, int32_t *ct_len,
            uint8_t *useg, const uint8_t *own)
{
    /* own (NULL = every mask): evaluate only the input masks g with own[g] != 0 (a rank's row
     * block in the sharded restatement, tests/oracle_shard_ctx.py) */
    int nU = 0;
#pragma omp parallel reduction(+ : nU)
    {
        int64_t cap = 1024;
        int64_t *keys = (int64_t *)malloc((size_t)cap * sizeof(int64_t));
#pragma omp for schedule(dynamic, 16)
        for (int g = 0; g < M_in; g++) {
            if (!kept[g] || (own && !own[g])) continue;
            const int r = gidx[g];
            /* valid points (mask minus boundary, :105) and their (frame, mask) entries;
             * key = frame << 32 | label (the column value of pim, :108) */
            int64_t T = 0, nk = 0;
            for (int64_t k = off[g]; k < off[g + 1]; k++) {
                const int32_t p = pts[k];
                if (boundary[p]) continue;
                T++;
                const int64_t ne = pt_off[p + 1] - pt_off[p];
                if (nk + ne > cap) {
                    while (nk + ne > cap) cap *= 2;
                    keys = (int64_t *)realloc(keys, (size_t)cap * sizeof(int64_t));
                }
                for (int64_t e = pt_off[p]; e < pt_off[p + 1]; e++) {
                    const int32_t h = pt_ent[e];
                    keys[nk++] = ((int64_t)col[h] << 32) | (int64_t)((uint32_t)label[h]);
                }
            }
            qsort(keys, (size_t)nk, sizeof(int64_t), cmp_i64);
            int split_num = 0, visible_num = 0, n = 0;
            for (int64_t i = 0; i < nk;) {   /* one possibly visible frame (:110) at a time */
                const int c = (int)(keys[i] >> 32);
                int64_t j = i, nz = 0, bestc = -1;
                int best = -1;
                while (j < nk && (int)(keys[j] >> 32) == c) {
                    int64_t j1 = j;
                    while (j1 < nk && keys[j1] == keys[j]) j1++;
                    const int64_t cnt = j1 - j;
                    const int v = (int)(uint32_t)(keys[j] & 0xffffffff);
                    nz += cnt;
                    if (cnt > bestc) { bestc = cnt; best = v; }   /* ascending labels: first max = smallest id (:122-123) */
                    j = j1;
                }
                i = j;
                const int64_t c0 = T - nz;
                const double invisible_ratio = (double)c0 / (double)T;            /* :117 */
                if (1.0 - invisible_ratio < mask_visible_threshold && nz < 500) continue;  /* :119 */
                visible_num++;
                const double contained_ratio = (double)bestc / (double)nz;        /* :124 */
                if (contained_ratio > contained_threshold) {                      /* :125-128 */
                    /* global index of (frame c, id best): masks of frame c are consecutive */
                    int lo = 0, hi = M_in - 1, tgt = -1;
                    while (lo <= hi) {
                        const int mid = (lo + hi) / 2;
                        const int64_t km = ((int64_t)col[mid] << 32) | (int64_t)(uint32_t)label[mid];
                        const int64_t kk = ((int64_t)c << 32) | (int64_t)(uint32_t)best;
                        if (km == kk) { tgt = mid; break; }
                        if (km < kk) lo = mid + 1; else hi = mid - 1;
                    }
                    ct_frame[(size_t)r * F_cap + n] = c;
                    ct_tgt[(size_t)r * F_cap + n] = gidx[tgt];
                    n++;
                } else {
                    split_num++;                                                  /* :130 */
                }
            }
            ct_len[r] = n;
            useg[r] = (visible_num == 0 || (double)split_num / (double)visible_num > undersegment_filter_threshold);
            nU += useg[r];
        }
        free(keys);
    }
    return nU;
}

/* undo (construction.py:160-169): entries whose target is under-segmented disappear (the C bit
 * and, col(u) being that entry's frame, the VF bit); rows compacted in place */
void orcs_undo(int M, int F_cap, int32_t *ct_frame, int32_t *ct_tgt, int32_t *ct_len, const uint8_t *useg)
{
#pragma omp parallel for schedule(static)
    for (int r = 0; r < M; r++) {
        int n = 0;
        for (int k = 0; k < ct_len[r]; k++) {
            const size_t e = (size_t)r * F_cap + k;
            if (useg[ct_tgt[e]]) continue;
            ct_frame[(size_t)r * F_cap + n] = ct_frame[e];
            ct_tgt[(size_t)r * F_cap + n] = ct_tgt[e];
            n++;
        }
        ct_len[r] = n;
    }
}

/* ------------------------------------------------------------------------ */
/* S4 (construction.py:84-86): histogram over all ordered pairs (i, j), i == j
 * included, of O = popcount(VF_i & VF_j), from VF bit rows. */
/* rank / world: only the pairs (i, j >= i) with i = rank (mod world) — one rank's share in the
 * sharded restatement; the shares' histograms sum to the whole one */
void orcs_observer_hist(int M, int FW, const uint64_t *vf, uint64_t *hist, int F, int rank, int world)
{
    /* per row: first and last non-zero word; a pair whose word ranges do not overlap has O = 0 */
    int32_t *wlo = (int32_t *)malloc((size_t)(M > 0 ? M : 1) * sizeof(int32_t));
    int32_t *whi = (int32_t *)malloc((size_t)(M > 0 ? M : 1) * sizeof(int32_t));
    for (int i = 0; i < M; i++) {
        wlo[i] = FW;
        whi[i] = -1;
        for (int w = 0; w < FW; w++)
            if (vf[(size_t)i * FW + w]) {
                if (wlo[i] == FW) wlo[i] = w;
                whi[i] = w;
            }
    }
    memset(hist, 0, (size_t)(F + 1) * sizeof(uint64_t));
#pragma omp parallel
    {
        uint64_t *h = (uint64_t *)calloc((size_t)F + 1, sizeof(uint64_t));
#pragma omp for schedule(dynamic, 32)
        for (int i = 0; i < M; i++) {
            if (i % world != rank) continue;
            const uint64_t *a = vf + (size_t)i * FW;
            int o = 0;
            for (int w = 0; w < FW; w++) o += __builtin_popcountll(a[w]);
            h[o] += 1;                                   /* the diagonal */
            uint64_t zeros = 0;
            for (int j = i + 1; j < M; j++) {            /* (i, j) and (j, i) */
                const int lo = wlo[i] > wlo[j] ? wlo[i] : wlo[j];
                const int hi = whi[i] < whi[j] ? whi[i] : whi[j];
                if (lo > hi) { zeros += 2; continue; }
                const uint64_t *b = vf + (size_t)j * FW;
                o = 0;
                for (int w = lo; w <= hi; w++) o += __builtin_popcountll(a[w] & b[w]);
                h[o] += 2;
            }
            h[0] += zeros;
        }
#pragma omp critical
        for (int v = 0; v <= F; v++) hist[v] += h[v];
        free(h);
    }
    free(wlo);
    free(whi);
}

/* ------------------------------------------------------------------------ */
/* S6 on sparse nodes: VF bit rows [N0][FW] and sorted contained-mask rows (c_off, c_idx) over
 * Mn mask ids.  Per threshold (iterative_clustering.py:39-43):
 *   S[a,b] = |C_a ∩ C_b| by column expansion (only pairs with S >= 1 can pass the rate test
 *   when ct > 0; ct <= 0 falls back to every pair), O[a,b] = popcount(VF_a & VF_b);
 *   edge iff a != b, !(O < thr) and fl32(S / fl32(O + 1e-7)) >= fl32(ct) (:20-29);
 *   components by BFS from the smallest unseen node (nx.connected_components, :7);
 *   new node = OR of its members (node.py:33-34).
 * labels_out[t * N0 + i]: component of level-t node i; level_sizes[t]; final_label[i];
 * edges_out[t] = number of undirected edges.  Returns the number of final nodes; the final
 * VF rows and C rows are left in vf_out [K][FW] and (c_off_out, c_idx_out). */
/* optional edge sink of orcs_cluster (test infrastructure: tests/test_setorder_cpu.py feeds the per-iteration
 * edges to the set-order restatement): keys (t << 48) | (a << 24) | b, a < b, up to cap; the count is
 * the total even past cap */
static uint64_t *g_edge_sink;
static int64_t g_edge_cap, g_edge_n;
void orcs_set_edge_sink(uint64_t *buf, int64_t cap)
{
    g_edge_sink = buf;
    g_edge_cap = cap;
    g_edge_n = 0;
}
int64_t orcs_edge_sink_count(void) { return g_edge_n; }

int orcs_cluster(int N0, int FW, int Mn, const uint64_t *vf0, const int64_t *c_off0, const int32_t *c_idx0,
                 int n_thr, const float *thr, double ct, int32_t *labels_out, int32_t *level_sizes,
                 int32_t *final_label, int64_t *edges_out, uint64_t *vf_out, int64_t *c_off_out, int32_t *c_idx_out)
{
    int N = N0;
    uint64_t *vf = (uint64_t *)malloc((size_t)(N0 > 0 ? N0 : 1) * FW * 8 + 8);
    memcpy(vf, vf0, (size_t)N0 * FW * 8);
    int64_t *coff = (int64_t *)malloc((size_t)(N0 + 1) * sizeof(int64_t));
    memcpy(coff, c_off0, (size_t)(N0 + 1) * sizeof(int64_t));
    int32_t *cidx = (int32_t *)malloc((size_t)(c_off0[N0] + 1) * sizeof(int32_t));
    memcpy(cidx, c_idx0, (size_t)c_off0[N0] * sizeof(int32_t));
    for (int i = 0; i < N0; i++) final_label[i] = i;
    const float ctf = (float)ct;
    const int dense = !(ct > 0.0);
    level_sizes[0] = N;
    int nthreads = 1;
#ifdef _OPENMP
    nthreads = omp_get_max_threads();
#endif
    int64_t *tedge_n = (int64_t *)calloc((size_t)nthreads, sizeof(int64_t));
    int64_t **tedges = (int64_t **)calloc((size_t)nthreads, sizeof(int64_t *));
    int64_t *tcap = (int64_t *)calloc((size_t)nthreads, sizeof(int64_t));
    for (int t = 0; t < n_thr; t++) {
        const float th = thr[t];
        /* column lists: nodes containing mask m, ascending */
        int64_t *moff = (int64_t *)calloc((size_t)Mn + 1, sizeof(int64_t));
        for (int64_t e = 0; e < coff[N]; e++) moff[cidx[e] + 1]++;
        for (int m = 0; m < Mn; m++) moff[m + 1] += moff[m];
        int32_t *mnodes = (int32_t *)malloc((size_t)(moff[Mn] + 1) * sizeof(int32_t));
        int64_t *mfill = (int64_t *)malloc((size_t)(Mn + 1) * sizeof(int64_t));
        memcpy(mfill, moff, (size_t)(Mn + 1) * sizeof(int64_t));
        for (int a = 0; a < N; a++)
            for (int64_t e = coff[a]; e < coff[a + 1]; e++) mnodes[mfill[cidx[e]]++] = a;
        free(mfill);
        for (int k = 0; k < nthreads; k++) tedge_n[k] = 0;
#pragma omp parallel
        {
            int tid = 0;
#ifdef _OPENMP
            tid = omp_get_thread_num();
#endif
            int32_t *cnt = (int32_t *)calloc((size_t)N + 1, sizeof(int32_t));
            int32_t *touched = (int32_t *)malloc((size_t)(N + 1) * sizeof(int32_t));
#pragma omp for schedule(dynamic, 16)
            for (int a = 0; a < N; a++) {
                int nt = 0;
                if (dense) {
                    for (int b = a + 1; b < N; b++) touched[nt++] = b;
                } else {
                    for (int64_t e = coff[a]; e < coff[a + 1]; e++) {
                        const int m = cidx[e];
                        for (int64_t q = moff[m]; q < moff[m + 1]; q++) {
                            const int b = mnodes[q];
                            if (b <= a) continue;
                            if (cnt[b]++ == 0) touched[nt++] = b;
                        }
                    }
                }
                const uint64_t *va = vf + (size_t)a * FW;
                for (int x = 0; x < nt; x++) {
                    const int b = touched[x];
                    const int s = cnt[b];
                    cnt[b] = 0;
                    const uint64_t *vb = vf + (size_t)b * FW;
                    int o = 0;
                    for (int w = 0; w < FW; w++) o += __builtin_popcountll(va[w] & vb[w]);
                    volatile float of = (float)o;
                    if (of < th) continue;                     /* disconnect (:26) */
                    volatile float den = of + 1e-7f;           /* observer_nums + 1e-7 (:23) */
                    volatile float rate = (float)s / den;
                    if (!(rate >= ctf)) continue;              /* :28 */
                    if (tedge_n[tid] == tcap[tid]) {
                        tcap[tid] = tcap[tid] ? 2 * tcap[tid] : 4096;
                        tedges[tid] = (int64_t *)realloc(tedges[tid], (size_t)tcap[tid] * sizeof(int64_t));
                    }
                    tedges[tid][tedge_n[tid]++] = ((int64_t)a << 32) | (int64_t)b;
                }
            }
            free(cnt);
            free(touched);
        }
        free(moff);
        free(mnodes);
        /* adjacency CSR (both directions, ascending neighbours) */
        int64_t E = 0;
        for (int k = 0; k < nthreads; k++) E += tedge_n[k];
        edges_out[t] = E;
        if (g_edge_sink)
            for (int k = 0; k < nthreads; k++)
                for (int64_t x = 0; x < tedge_n[k]; x++, g_edge_n++)
                    if (g_edge_n < g_edge_cap)
                        g_edge_sink[g_edge_n] = ((uint64_t)t << 48) | ((uint64_t)(tedges[k][x] >> 32) << 24) |
                                                (uint64_t)(tedges[k][x] & 0xffffffff);
        int64_t *aoff = (int64_t *)calloc((size_t)N + 1, sizeof(int64_t));
        for (int k = 0; k < nthreads; k++)
            for (int64_t x = 0; x < tedge_n[k]; x++) {
                aoff[(tedges[k][x] >> 32) + 1]++;
                aoff[(tedges[k][x] & 0xffffffff) + 1]++;
            }
        for (int i = 0; i < N; i++) aoff[i + 1] += aoff[i];
        int32_t *adj = (int32_t *)malloc((size_t)(2 * E + 1) * sizeof(int32_t));
        int64_t *afill = (int64_t *)malloc((size_t)(N + 1) * sizeof(int64_t));
        memcpy(afill, aoff, (size_t)(N + 1) * sizeof(int64_t));
        for (int k = 0; k < nthreads; k++)
            for (int64_t x = 0; x < tedge_n[k]; x++) {
                const int a = (int)(tedges[k][x] >> 32), b = (int)(tedges[k][x] & 0xffffffff);
                adj[afill[a]++] = b;
                adj[afill[b]++] = a;
            }
        free(afill);
        /* components: BFS from the smallest unseen node, labels in discovery order of the roots */
        int32_t *lab = labels_out + (size_t)t * N0;
        for (int i = 0; i < N; i++) lab[i] = -1;
        int32_t *queue = (int32_t *)malloc((size_t)(N + 1) * sizeof(int32_t));
        int K = 0;
        for (int s = 0; s < N; s++) {
            if (lab[s] >= 0) continue;
            int qh = 0, qt = 0;
            queue[qt++] = s;
            lab[s] = K;
            while (qh < qt) {
                const int u = queue[qh++];
                for (int64_t e = aoff[u]; e < aoff[u + 1]; e++)
                    if (lab[adj[e]] < 0) { lab[adj[e]] = K; queue[qt++] = adj[e]; }
            }
            K++;
        }
        free(queue);
        free(aoff);
        free(adj);
        /* merge (node.py:27-36): OR of VF rows, sorted union of C rows */
        uint64_t *nvf = (uint64_t *)calloc((size_t)(K > 0 ? K : 1) * FW, 8);
        int64_t *ncoff = (int64_t *)calloc((size_t)K + 1, sizeof(int64_t));
        int64_t *moff2 = (int64_t *)calloc((size_t)K + 1, sizeof(int64_t));
        for (int i = 0; i < N; i++) moff2[lab[i] + 1]++;
        for (int k = 0; k < K; k++) moff2[k + 1] += moff2[k];
        int32_t *mem = (int32_t *)malloc((size_t)(N + 1) * sizeof(int32_t));
        int64_t *mf = (int64_t *)malloc((size_t)(K + 1) * sizeof(int64_t));
        memcpy(mf, moff2, (size_t)(K + 1) * sizeof(int64_t));
        for (int i = 0; i < N; i++) mem[mf[lab[i]]++] = i;
        free(mf);
        int32_t **rows = (int32_t **)malloc((size_t)(K > 0 ? K : 1) * sizeof(int32_t *));
#pragma omp parallel
        {
            int32_t *buf = NULL;
            int64_t bcap = 0;
#pragma omp for schedule(dynamic, 16)
            for (int k = 0; k < K; k++) {
                int64_t tot = 0;
                for (int64_t q = moff2[k]; q < moff2[k + 1]; q++) {
                    const int i = mem[q];
                    for (int w = 0; w < FW; w++) nvf[(size_t)k * FW + w] |= vf[(size_t)i * FW + w];
                    tot += coff[i + 1] - coff[i];
                }
                if (tot > bcap) { bcap = tot; buf = (int32_t *)realloc(buf, (size_t)bcap * sizeof(int32_t)); }
                int64_t n = 0;
                for (int64_t q = moff2[k]; q < moff2[k + 1]; q++) {
                    const int i = mem[q];
                    for (int64_t e = coff[i]; e < coff[i + 1]; e++) buf[n++] = cidx[e];
                }
                /* sort + unique (insertion sort: rows are short, members already sorted) */
                for (int64_t x = 1; x < n; x++) {
                    const int32_t v = buf[x];
                    int64_t y = x - 1;
                    while (y >= 0 && buf[y] > v) { buf[y + 1] = buf[y]; y--; }
                    buf[y + 1] = v;
                }
                int64_t u = 0;
                for (int64_t x = 0; x < n; x++)
                    if (u == 0 || buf[x] != buf[u - 1]) buf[u++] = buf[x];
                rows[k] = (int32_t *)malloc((size_t)(u + 1) * sizeof(int32_t));
                memcpy(rows[k], buf, (size_t)u * sizeof(int32_t));
                ncoff[k + 1] = u;
            }
            free(buf);
        }
        for (int k = 0; k < K; k++) ncoff[k + 1] += ncoff[k];
        int32_t *ncidx = (int32_t *)malloc((size_t)(ncoff[K] + 1) * sizeof(int32_t));
        for (int k = 0; k < K; k++) {
            memcpy(ncidx + ncoff[k], rows[k], (size_t)(ncoff[k + 1] - ncoff[k]) * sizeof(int32_t));
            free(rows[k]);
        }
        free(rows);
        free(mem);
        free(moff2);
        free(vf); free(coff); free(cidx);
        vf = nvf; coff = ncoff; cidx = ncidx;
        for (int i = 0; i < N0; i++) final_label[i] = lab[final_label[i]];
        N = K;
        level_sizes[t + 1] = N;
    }
    memcpy(vf_out, vf, (size_t)N * FW * 8);
    memcpy(c_off_out, coff, (size_t)(N + 1) * sizeof(int64_t));
    memcpy(c_idx_out, cidx, (size_t)coff[N] * sizeof(int32_t));
    for (int k = 0; k < nthreads; k++) free(tedges[k]);
    free(tedges); free(tedge_n); free(tcap);
    free(vf); free(coff); free(cidx);
    return N;
}

/* ------------------------------------------------------------------------ */
/* The edges of one S6 iteration (graph/iterative_clustering.py:20-29) for the rows a with
 * a = rank (mod world), b > a: the same rule as orcs_cluster.  Writes up to cap (a, b) pairs
 * into edges (a << 32 | b); returns the number of edges (callers retry with a larger cap). */
int64_t orcs_level_edges(int N, int FW, int Mn, const uint64_t *vf, const int64_t *coff, const int32_t *cidx,
                         float th, double ct, int rank, int world, int64_t *edges, int64_t cap)
{
    const float ctf = (float)ct;
    const int dense = !(ct > 0.0);
    int64_t *moff = (int64_t *)calloc((size_t)Mn + 1, sizeof(int64_t));
    for (int64_t e = 0; e < coff[N]; e++) moff[cidx[e] + 1]++;
    for (int m = 0; m < Mn; m++) moff[m + 1] += moff[m];
    int32_t *mnodes = (int32_t *)malloc((size_t)(moff[Mn] + 1) * sizeof(int32_t));
    int64_t *mfill = (int64_t *)malloc((size_t)(Mn + 1) * sizeof(int64_t));
    memcpy(mfill, moff, (size_t)(Mn + 1) * sizeof(int64_t));
    for (int a = 0; a < N; a++)
        for (int64_t e = coff[a]; e < coff[a + 1]; e++) mnodes[mfill[cidx[e]]++] = a;
    free(mfill);
    int32_t *cnt = (int32_t *)calloc((size_t)N + 1, sizeof(int32_t));
    int32_t *touched = (int32_t *)malloc((size_t)(N + 1) * sizeof(int32_t));
    int64_t ne = 0;
    for (int a = rank; a < N; a += world) {
        int nt = 0;
        if (dense) {
            for (int b = a + 1; b < N; b++) touched[nt++] = b;
        } else {
            for (int64_t e = coff[a]; e < coff[a + 1]; e++)
                for (int64_t q = moff[cidx[e]]; q < moff[cidx[e] + 1]; q++) {
                    const int b = mnodes[q];
                    if (b > a && cnt[b]++ == 0) touched[nt++] = b;
                }
        }
        for (int x = 0; x < nt; x++) {
            const int b = touched[x];
            const int sv = cnt[b];
            cnt[b] = 0;
            int o = 0;
            for (int w = 0; w < FW; w++) o += __builtin_popcountll(vf[(size_t)a * FW + w] & vf[(size_t)b * FW + w]);
            volatile float of = (float)o;
            if (of < th) continue;
            volatile float den = of + 1e-7f;
            volatile float rate = (float)sv / den;
            if (!(rate >= ctf)) continue;
            if (ne < cap) edges[ne] = ((int64_t)a << 32) | (int64_t)b;
            ne++;
        }
    }
    free(cnt); free(touched); free(moff); free(mnodes);
    return ne;
}
