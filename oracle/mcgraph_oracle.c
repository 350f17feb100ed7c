/*
 * mcgraph_oracle.c — CPU restatement of MaskClustering's view-consensus graph
 * stages S2–S6.  TEST INFRASTRUCTURE ONLY: this file is the checker that the
 * HIP path is compared against (tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py).  It is never linked into, loaded by or called
 * from the product library.
 *
 * It follows the reference's structure on purpose (dense point-in-mask matrix,
 * per-mask loops, dense N×N observer/supporter counts, BFS components), with
 * Python list scans replaced by lookup tables.  Parity is pinned by the golden
 * fixtures in tests/golden/ that were produced by running the reference itself
 * (tests/golden/make_golden.py).
 *
 * Float semantics: all S3 ratio tests in double like
 * numpy/Python; the S6 rate and comparisons in float32 like torch; the S4
 * percentile in float32 like numpy 2.x.  Build with -ffp-contract=off.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* S2  build_point_in_mask_matrix  (graph/construction.py:22-64)             */
/* ------------------------------------------------------------------------ */
/* Input masks are the per-frame mask dicts flattened in frame order, ids in the
 * dict's (ascending) order.  A frame whose union of mask sets is empty is
 * skipped entirely (construction.py:50-51): its masks get kept[g] = 0 and are
 * not part of the global list (construction.py:60).
 * pim[p*F + c] = id if p lies in exactly one mask of frame c (construction.py:58,61)
 * pfm[p*F + c] = 1 if p lies in any mask of frame c      (construction.py:52)
 * boundary[p]  = 1 if p lies in >= 2 masks of some frame  (construction.py:56,62)
 * Returns the number of kept (global) masks. */
int orc_s2(int64_t P, int F, int M_in, const int32_t *col, const int32_t *label,
           const int64_t *off, const int32_t *pts, uint8_t *kept, uint16_t *pim,
           uint8_t *pfm, uint8_t *boundary)
{
    memset(pim, 0, (size_t)P * F * sizeof(uint16_t));
    memset(pfm, 0, (size_t)P * F);
    memset(boundary, 0, (size_t)P);
    uint8_t *multi = (uint8_t *)calloc((size_t)P, 1); /* per-frame "appeared" */
    int M = 0;
    int g = 0;
    while (g < M_in) {
        int c = col[g];
        int g1 = g;
        int64_t frame_pts = 0;
        while (g1 < M_in && col[g1] == c) { frame_pts += off[g1 + 1] - off[g1]; g1++; }
        if (frame_pts == 0) {           /* construction.py:50-51 */
            for (int h = g; h < g1; h++) kept[h] = 0;
            g = g1;
            continue;
        }
        /* appeared_point_ids / frame_boundary_point_index (construction.py:53-59) */
        for (int h = g; h < g1; h++) {
            kept[h] = 1;
            M++;
            for (int64_t k = off[h]; k < off[h + 1]; k++) {
                int64_t p = pts[k];
                pfm[p * F + c] = 1;
                if (multi[p]) multi[p] = 2;      /* intersection with appeared */
                else multi[p] = 1;
                pim[p * F + c] = (uint16_t)label[h];
            }
        }
        for (int h = g; h < g1; h++) {
            for (int64_t k = off[h]; k < off[h + 1]; k++) {
                int64_t p = pts[k];
                if (multi[p] == 2) { pim[p * F + c] = 0; boundary[p] = 1; }  /* :61-62 */
            }
        }
        for (int h = g; h < g1; h++)
            for (int64_t k = off[h]; k < off[h + 1]; k++) multi[pts[k]] = 0;
        g = g1;
    }
    free(multi);
    return M;
}

/* ------------------------------------------------------------------------ */
/* S3  process_one_mask / process_masks  (graph/construction.py:98-170)      */
/* ------------------------------------------------------------------------ */
/* Global masks only (kept).  Outputs:
 *   vf[g*F + c]   visible_frame (0/1) after the under-segmentation undo
 *   ctgt[g*F + c] the contained mask index in frame c or -1 (the single C-bit
 *                 of row g in frame c, construction.py:126-128), after undo
 *   useg[g]       1 if under-segmented (construction.py:132,156-158)
 * Returns the number of under-segmented masks. */
int orc_s3(int64_t P, int F, int M, const int32_t *col, const int32_t *label,
           const int64_t *off, const int32_t *pts, const uint16_t *pim,
           const uint8_t *boundary, double mask_visible_threshold,
           double contained_threshold, double undersegment_filter_threshold,
           uint8_t *vf, int32_t *ctgt, uint8_t *useg)
{
    (void)P;
    /* (frame col, label) -> global index: replaces list.index (construction.py:127,157) */
    int32_t *lut = (int32_t *)malloc((size_t)F * 65536 * sizeof(int32_t));
    for (size_t i = 0; i < (size_t)F * 65536; i++) lut[i] = -1;
    for (int g = 0; g < M; g++) lut[(size_t)col[g] * 65536 + label[g]] = g;

    int64_t *cnt = (int64_t *)calloc(65536, sizeof(int64_t));
    int32_t *touched = (int32_t *)malloc(65536 * sizeof(int32_t));
    int64_t *vrows = NULL;
    int64_t vcap = 0;
    int nU = 0;
    memset(vf, 0, (size_t)M * F);
    for (size_t i = 0; i < (size_t)M * F; i++) ctgt[i] = -1;

    for (int g = 0; g < M; g++) {
        /* valid_mask_point_cloud = mask - boundary (construction.py:105) */
        int64_t T = 0;
        int64_t n = off[g + 1] - off[g];
        if (n > vcap) { vcap = n; vrows = (int64_t *)realloc(vrows, (size_t)vcap * sizeof(int64_t)); }
        for (int64_t k = off[g]; k < off[g + 1]; k++)
            if (!boundary[pts[k]]) vrows[T++] = pts[k];
        int split_num = 0, visible_num = 0;
        for (int c = 0; c < F; c++) {
            /* possibly_visible_frames: column sum > 0 (construction.py:110) */
            int ntouch = 0;
            int64_t c0 = 0;
            for (int64_t i = 0; i < T; i++) {
                uint16_t v = pim[vrows[i] * F + c];
                if (v == 0) { c0++; continue; }
                if (cnt[v] == 0) touched[ntouch++] = v;
                cnt[v]++;
            }
            if (ntouch == 0) continue;
            int64_t total = T;                     /* np.sum(mask_id_count) */
            int64_t nz = total - c0;
            double invisible_ratio = (double)c0 / (double)total;          /* :117 */
            if (1.0 - invisible_ratio < mask_visible_threshold && nz < 500) { /* :119 */
                for (int i = 0; i < ntouch; i++) cnt[touched[i]] = 0;
                continue;
            }
            visible_num++;
            /* argmax over ids >= 1, first (smallest id) on ties (:122-123) */
            int best = -1;
            int64_t bestc = -1;
            for (int i = 0; i < ntouch; i++) {
                int v = touched[i];
                if (cnt[v] > bestc || (cnt[v] == bestc && v < best)) { bestc = cnt[v]; best = v; }
            }
            double contained_ratio = (double)bestc / (double)nz;           /* :124 */
            if (contained_ratio > contained_threshold) {                   /* :125-128 */
                vf[(size_t)g * F + c] = 1;
                ctgt[(size_t)g * F + c] = lut[(size_t)c * 65536 + best];
            } else {
                split_num++;                                               /* :130 */
            }
            for (int i = 0; i < ntouch; i++) cnt[touched[i]] = 0;
        }
        /* :132 */
        if (visible_num == 0 || (double)split_num / (double)visible_num > undersegment_filter_threshold) {
            useg[g] = 1;
            nU++;
        } else {
            useg[g] = 0;
        }
    }
    /* under-segmentation undo (construction.py:164-169) */
    for (int r = 0; r < M; r++) {
        for (int c = 0; c < F; c++) {
            int32_t t = ctgt[(size_t)r * F + c];
            if (t >= 0 && useg[t]) {
                ctgt[(size_t)r * F + c] = -1;
                vf[(size_t)r * F + c] = 0;   /* visible_frames[rows, col(u)] = 0, col(u) == c */
            }
        }
    }
    free(lut); free(cnt); free(touched); free(vrows);
    return nU;
}

/* ------------------------------------------------------------------------ */
/* S4  get_observer_num_thresholds  (graph/construction.py:80-96)            */
/* ------------------------------------------------------------------------ */
/* hist[v] = #ordered pairs (i, j), i==j included, with (VF·VFᵀ)[i,j] == v, v in [0,F]. */
void orc_observer_hist(int M, int F, const uint8_t *vf, uint64_t *hist)
{
    int FW = (F + 63) / 64;
    uint64_t *bits = (uint64_t *)calloc((size_t)M * FW, sizeof(uint64_t));
    for (int g = 0; g < M; g++)
        for (int c = 0; c < F; c++)
            if (vf[(size_t)g * F + c]) bits[(size_t)g * FW + c / 64] |= 1ull << (c % 64);
    memset(hist, 0, (size_t)(F + 1) * sizeof(uint64_t));
#pragma omp parallel
    {
        uint64_t *h = (uint64_t *)calloc((size_t)F + 1, sizeof(uint64_t));
#pragma omp for schedule(dynamic, 16)
        for (int i = 0; i < M; i++) {
            const uint64_t *a = bits + (size_t)i * FW;
            for (int j = 0; j < M; j++) {
                const uint64_t *b = bits + (size_t)j * FW;
                int o = 0;
                for (int w = 0; w < FW; w++) o += __builtin_popcountll(a[w] & b[w]);
                h[o]++;
            }
        }
#pragma omp critical
        for (int v = 0; v <= F; v++) hist[v] += h[v];
        free(h);
    }
    free(bits);
}

/* k-th (0-based) order statistic of the multiset of positive observer counts */
static float order_stat(const uint64_t *hist, int F, uint64_t k)
{
    uint64_t acc = 0;
    for (int v = 1; v <= F; v++) {
        acc += hist[v];
        if (k < acc) return (float)v;
    }
    return (float)F;
}

/* np.percentile(x, p) for float32 x, numpy 2.x "linear" method
 * (numpy/lib/_function_base_impl.py: percentile q = p / float32(100);
 *  _compute_virtual_index (n-1)*q in float32; _get_indexes; _get_gamma;
 *  _lerp with the t >= 0.5 branch). */
static float np2_percentile_f32(const uint64_t *hist, int F, uint64_t n, int p)
{
    volatile float q = (float)p / 100.0f;
    volatile float nm1 = (float)(n - 1);
    volatile float vi = nm1 * q;
    int64_t prev, next;
    if (vi >= nm1) {                      /* indexes_above_bounds -> -1 (last) */
        prev = -1; next = -1;
    } else {
        prev = (int64_t)floorf(vi);
        next = prev + 1;
        if (vi < 0) { prev = 0; next = 0; }
    }
    uint64_t ip = prev < 0 ? n - 1 : (uint64_t)prev;
    uint64_t in = next < 0 ? n - 1 : (uint64_t)next;
    volatile float gamma = (float)((double)vi - (double)prev);
    volatile float a = order_stat(hist, F, ip);
    volatile float b = order_stat(hist, F, in);
    volatile float diff = b - a;
    volatile float t1 = diff * gamma;
    volatile float r = a + t1;
    if (gamma >= 0.5f) {
        volatile float omg = 1.0f - gamma;
        volatile float t2 = diff * omg;
        r = b - t2;
    }
    return r;
}

/* Fills thr[0..n) and is_int[] (1 where the reference substitutes the Python
 * int 1, construction.py:94).  Returns n, or -1 where the reference raises
 * (no positive observer count: np.percentile on an empty array). */
int orc_thresholds(const uint64_t *hist, int F, float *thr, int32_t *is_int)
{
    uint64_t n = 0;
    for (int v = 1; v <= F; v++) n += hist[v];
    if (n == 0) return -1;
    int k = 0;
    for (int p = 95; p > -5; p -= 5) {                  /* construction.py:88 */
        float t = np2_percentile_f32(hist, F, n, p);
        int isint = 0;
        if (t <= 1.0f) {                                /* :90-94 */
            if (p < 50) break;
            t = 1.0f;
            isint = 1;
        }
        thr[k] = t;
        is_int[k] = isint;
        k++;
    }
    return k;
}

/* ------------------------------------------------------------------------ */
/* S6  update_graph / cluster_into_new_nodes / iterative_clustering          */
/*     (graph/iterative_clustering.py:5-43), Node merge (graph/node.py:24-37) */
/* ------------------------------------------------------------------------ */
/* Nodes start as the N0 initial nodes given by their VF (F bytes) and C
 * (M bytes) rows.  For each threshold: observer O = VF·VFᵀ and supporter
 * S = C·Cᵀ (exact integer counts, like the fp32 SGEMMs), edge iff i != j,
 * !(O < thr) and fl32(S / fl32(O + 1e-7f)) >= fl32(ct)  (:20-29, torch float32
 * semantics); components in ascending order of their smallest member (networkx
 * BFS from the smallest unseen node, :7); new node = OR of members (node.py:33-34).
 * labels_out[t * N0 + i] = component of level-t node i (only the first N_t
 * entries of each row are meaningful).  final_label[i] = final node of initial
 * node i.  Returns the number of final nodes. */
int orc_cluster(int N0, int F, int M, const uint8_t *vf0, const uint8_t *cm0,
                int n_thr, const float *thr, double ct, int32_t *labels_out,
                int32_t *level_sizes, int32_t *final_label, uint8_t *vf_out,
                uint8_t *cm_out)
{
    int FW = (F + 63) / 64, MW = (M + 63) / 64;
    uint64_t *vf = (uint64_t *)calloc((size_t)N0 * FW, 8);
    uint64_t *cm = (uint64_t *)calloc((size_t)N0 * MW, 8);
    for (int i = 0; i < N0; i++) {
        for (int c = 0; c < F; c++) if (vf0[(size_t)i * F + c]) vf[(size_t)i * FW + c / 64] |= 1ull << (c % 64);
        for (int m = 0; m < M; m++) if (cm0[(size_t)i * M + m]) cm[(size_t)i * MW + m / 64] |= 1ull << (m % 64);
    }
    int N = N0;
    for (int i = 0; i < N0; i++) final_label[i] = i;
    float ctf = (float)ct;
    int32_t *parent = (int32_t *)malloc((size_t)N0 * sizeof(int32_t));
    int32_t *adj_deg = (int32_t *)malloc((size_t)N0 * sizeof(int32_t));
    uint8_t *adj = NULL;
    level_sizes[0] = N;
    for (int t = 0; t < n_thr; t++) {
        float th = thr[t];
        free(adj);
        adj = (uint8_t *)calloc((size_t)N * N, 1);
#pragma omp parallel for schedule(dynamic, 8)
        for (int i = 0; i < N; i++) {
            const uint64_t *vi = vf + (size_t)i * FW, *ci = cm + (size_t)i * MW;
            for (int j = i + 1; j < N; j++) {
                const uint64_t *vj = vf + (size_t)j * FW, *cj = cm + (size_t)j * MW;
                int o = 0, s = 0;
                for (int w = 0; w < FW; w++) o += __builtin_popcountll(vi[w] & vj[w]);
                volatile float of = (float)o;
                if (of < th) continue;                       /* disconnect (:26) */
                for (int w = 0; w < MW; w++) s += __builtin_popcountll(ci[w] & cj[w]);
                volatile float den = of + 1e-7f;             /* observer_nums + 1e-7 (:23) */
                volatile float rate = (float)s / den;
                if (rate >= ctf) { adj[(size_t)i * N + j] = 1; adj[(size_t)j * N + i] = 1; }  /* :28 */
            }
        }
        (void)adj_deg;
        /* connected components, ordered by smallest member (BFS from min unseen) */
        for (int i = 0; i < N; i++) parent[i] = -1;
        int K = 0;
        int32_t *queue = (int32_t *)malloc((size_t)N * sizeof(int32_t));
        for (int s = 0; s < N; s++) {
            if (parent[s] >= 0) continue;
            int qh = 0, qt = 0;
            queue[qt++] = s;
            parent[s] = K;
            while (qh < qt) {
                int u = queue[qh++];
                const uint8_t *row = adj + (size_t)u * N;
                for (int v = 0; v < N; v++)
                    if (row[v] && parent[v] < 0) { parent[v] = K; queue[qt++] = v; }
            }
            K++;
        }
        free(queue);
        memcpy(labels_out + (size_t)t * N0, parent, (size_t)N * sizeof(int32_t));
        /* merge (node.py:27-36): OR of members */
        uint64_t *nvf = (uint64_t *)calloc((size_t)K * FW, 8);
        uint64_t *ncm = (uint64_t *)calloc((size_t)K * MW, 8);
        for (int i = 0; i < N; i++) {
            int k = parent[i];
            for (int w = 0; w < FW; w++) nvf[(size_t)k * FW + w] |= vf[(size_t)i * FW + w];
            for (int w = 0; w < MW; w++) ncm[(size_t)k * MW + w] |= cm[(size_t)i * MW + w];
        }
        free(vf); free(cm);
        vf = nvf; cm = ncm;
        for (int i = 0; i < N0; i++) final_label[i] = parent[final_label[i]];
        N = K;
        level_sizes[t + 1] = N;
    }
    for (int k = 0; k < N; k++) {
        for (int c = 0; c < F; c++) vf_out[(size_t)k * F + c] = (vf[(size_t)k * FW + c / 64] >> (c % 64)) & 1;
        for (int m = 0; m < M; m++) cm_out[(size_t)k * M + m] = (cm[(size_t)k * MW + m / 64] >> (m % 64)) & 1;
    }
    free(adj); free(vf); free(cm); free(parent); free(adj_deg);
    return N;
}

int orc_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* thread count of the OpenMP loops above (bench.py's single-thread / all-core baselines) */
void orc_set_num_threads(int n)
{
#ifdef _OPENMP
    omp_set_num_threads(n > 0 ? n : 1);
#else
    (void)n;
#endif
}
