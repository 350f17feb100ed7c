/*
 * s1_oracle.c — CPU restatement of MaskClustering's per-frame mask
 * back-projection (stage S1): utils/mask_backprojection.py:70-151 together
 * with utils/geometry.py:9-24 (denoise).  TEST INFRASTRUCTURE ONLY: this is
 * the checker the HIP path is compared against (tests/, smoke(), bench.py's
 * cpu_baseline leg).  It is never linked into or called by the product.
 *
 * PARITY UNPINNED for the library arithmetic.  It lives in third-party code
 * that is absent from /root/reference and from this container:
 *   Open3D (version unpinned, requirements.txt:2): PointCloud.create_from_depth_image
 *     + transform (mask_backprojection.py:22-23), voxel_down_sample (:105),
 *     cluster_dbscan / select_by_index / remove_statistical_outlier
 *     (geometry.py:10,20,22);
 *   pytorch3d 0.7.3 (dockerfile:39): ops.ball_query (mask_backprojection.py:38).
 * The reference's own glue around those calls (:70-151) is pinned by fixtures
 * made by running it with these restated library ops (tests/golden/make_s1_golden.py).
 * Choices made where the libraries' result is not determined by their
 * published algorithm:
 *   (u1) Eigen evaluation order of the 4x4 transform without FMA:
 *        ((T[r][0]x + T[r][1]y) + T[r][2]z) + T[r][3], then / w.
 *   (u2) voxel_down_sample's output order is std::unordered_map iteration order
 *        (hash and libstdc++ dependent).  We use first-occurrence order (the
 *        order of the first pixel, row-major, that falls in each voxel).  The
 *        per-voxel sum itself is Open3D's: sequential in input order, / count.
 *   (u3) KD-tree squared distances as nanoflann's L2 adaptor for 3-D:
 *        ((0 + dx*dx) + dy*dy) + dz*dz in double; radius test d2 < eps*eps.
 *   (u4) pytorch3d's float32 dist2 loop is contracted to FMA by nvcc:
 *        d2 = fmaf(dz, dz, fmaf(dy, dy, dx*dx)); radius2 = float(r) * float(r).
 * Output sets are order-free; (u2) only matters at DBSCAN border ties and in the
 * last bits of the outlier statistics.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    double depth_trunc;            /* DEPTH_TRUNC = 20             mask_backprojection.py:13,22,44 */
    double voxel_size;             /* DISTANCE_THRESHOLD = 0.01    :10,105 */
    double dbscan_eps;             /* 0.04                         geometry.py:10 */
    double component_min_fraction; /* 0.2                          geometry.py:16 */
    double sor_std_ratio;          /* 2.0                          geometry.py:22 */
    double ball_radius;            /* DISTANCE_THRESHOLD (float32) :38 */
    double coverage_threshold;     /* COVERAGE_THRESHOLD = 0.3     :8,145 */
    int32_t dbscan_min_points;     /* 4                            geometry.py:10 */
    int32_t sor_neighbors;         /* 20                           geometry.py:22 */
    int32_t ball_k;                /* K = 20                       :38 */
    int32_t few_points;            /* FEW_POINTS_THRESHOLD = 25    :11,101,109 */
} orc_bp_params;

/* per candidate mask (every id != 0 of the image, ascending) */
enum { ST_ID = 0, ST_NPIX, ST_NVOX, ST_NDB, ST_NSOR, ST_NCAND, ST_NCOV, ST_NNBR, ST_KEPT, ST_NSTAT };

/* ---- (a1) backproject (:17-24): Open3D depth -> camera -> world ----------- */
static void world_point(const double *K, const double *T, int u, int v, float d, double out[3])
{
    const double z = (double)d;
    volatile double x = ((double)u - K[2]) * z;
    x = x / K[0];
    volatile double y = ((double)v - K[3]) * z;
    y = y / K[1];
    double r[4];
    for (int k = 0; k < 4; k++) {
        volatile double a = T[4 * k] * x;
        volatile double b = T[4 * k + 1] * y;
        volatile double c = T[4 * k + 2] * z;
        volatile double s = a + b;
        s = s + c;
        s = s + T[4 * k + 3];
        r[k] = s;
    }
    for (int k = 0; k < 3; k++) out[k] = r[k] / r[3];
}

/* built with -ffp-contract=off and without -ffast-math on x86-64 (SSE2 doubles), so this is
 * evaluated exactly as written: three rounded products, two rounded sums, in this order */
static inline double d2_f64(const double *a, const double *b)
{
    const double dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    return ((dx * dx) + (dy * dy)) + (dz * dz);
}

/* ---- (a3) voxel_down_sample (:105), first-occurrence order (u2) ---------- */
static int voxel_down(const double *pts, int n, double vs, double *out)
{
    double mn[3] = {pts[0], pts[1], pts[2]};
    for (int i = 1; i < n; i++)
        for (int r = 0; r < 3; r++)
            if (pts[3 * i + r] < mn[r]) mn[r] = pts[3 * i + r];
    double vmin[3];
    for (int r = 0; r < 3; r++) vmin[r] = mn[r] - vs * 0.5;
    int cap = 1;
    while (cap < 2 * n) cap <<= 1;
    int64_t *keys = (int64_t *)malloc((size_t)cap * sizeof(int64_t));
    int32_t *vid = (int32_t *)malloc((size_t)cap * sizeof(int32_t));
    for (int i = 0; i < cap; i++) keys[i] = -1;
    double *sum = (double *)calloc((size_t)3 * n, sizeof(double));
    int32_t *cnt = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    int nv = 0;
    for (int i = 0; i < n; i++) {
        int64_t ix[3];
        for (int r = 0; r < 3; r++) {
            volatile double t = pts[3 * i + r] - vmin[r];
            t = t / vs;
            ix[r] = (int64_t)floor(t);
        }
        const int64_t key = (ix[0] << 42) | (ix[1] << 21) | ix[2];
        const uint64_t h = (uint64_t)key * 0x9E3779B97F4A7C15ull;
        int s = (int)(h >> 40) & (cap - 1);
        while (keys[s] != -1 && keys[s] != key) s = (s + 1) & (cap - 1);
        if (keys[s] == -1) {
            keys[s] = key;
            vid[s] = nv++;
        }
        const int v = vid[s];
        for (int r = 0; r < 3; r++) sum[3 * v + r] = sum[3 * v + r] + pts[3 * i + r];  /* AccumulatedPoint::AddPoint */
        cnt[v]++;
    }
    for (int v = 0; v < nv; v++)
        for (int r = 0; r < 3; r++) out[3 * v + r] = sum[3 * v + r] / (double)cnt[v];  /* GetAveragePoint */
    free(keys); free(vid); free(sum); free(cnt);
    return nv;
}

/* ---- (a4) denoise (geometry.py:9-24) ------------------------------------ */
/* Open3D ClusterDBSCAN, literally: labels -2 unvisited / -1 noise; seeds in index
 * order; expansion from core points only; a noise point reached later becomes a
 * border point of the cluster that reaches it. */
static void dbscan(const double *p, int n, double eps, int minpts, int32_t *labels)
{
    const double e2 = eps * eps;
    int32_t *nbo = (int32_t *)malloc((size_t)(n + 1) * sizeof(int32_t));
    int64_t tot = 0, ncap = 16 * (int64_t)n + 16;
    int32_t *nb = (int32_t *)malloc((size_t)ncap * sizeof(int32_t));
    nbo[0] = 0;
    for (int i = 0; i < n; i++) {  /* every point's eps-neighbours (self included), ascending index */
        for (int j = 0; j < n; j++)
            if (d2_f64(p + 3 * i, p + 3 * j) < e2) {
                if (tot == ncap) {
                    ncap *= 2;
                    nb = (int32_t *)realloc(nb, (size_t)ncap * sizeof(int32_t));
                }
                nb[tot++] = j;
            }
        nbo[i + 1] = (int32_t)tot;
    }
    uint8_t *queued = (uint8_t *)calloc((size_t)n + 1, 1);
    int32_t *queue = (int32_t *)malloc((size_t)(n + 1) * sizeof(int32_t));
    for (int i = 0; i < n; i++) labels[i] = -2;
    int cl = 0;
    for (int idx = 0; idx < n; idx++) {
        if (labels[idx] != -2) continue;
        if (nbo[idx + 1] - nbo[idx] < minpts) {
            labels[idx] = -1;
            continue;
        }
        memset(queued, 0, (size_t)n);
        int qh = 0, qt = 0;
        queued[idx] = 1;
        for (int k = nbo[idx]; k < nbo[idx + 1]; k++)
            if (!queued[nb[k]]) { queued[nb[k]] = 1; queue[qt++] = nb[k]; }
        labels[idx] = cl;
        while (qh < qt) {
            const int q = queue[qh++];
            if (labels[q] == -1) labels[q] = cl;
            if (labels[q] != -2) continue;
            labels[q] = cl;
            if (nbo[q + 1] - nbo[q] >= minpts)
                for (int k = nbo[q]; k < nbo[q + 1]; k++)
                    if (!queued[nb[k]]) { queued[nb[k]] = 1; queue[qt++] = nb[k]; }
        }
        cl++;
    }
    free(nbo); free(nb); free(queued); free(queue);
}

/* remove_statistical_outlier(nb_neighbors, std_ratio) on the points idx[0..m):
 * keep[i] for i < m.  Returns the number kept. */
static int statistical_outlier(const double *p, const int32_t *idx, int m, int k, double std_ratio, uint8_t *keep)
{
    /* nb_neighbors < 1 is an illegal input to Open3D's RemoveStatisticalOutliers (the C-ABI rejects
       it with MC_ERR_UNSUPPORTED); nothing is kept here, and no d[kk - 1] read happens with kk = 0 */
    if (m == 0 || k < 1) return 0;
    const int kk = k < m ? k : m;                     /* nanoflann returns min(k, n) */
    double *avg = (double *)malloc((size_t)m * sizeof(double));
    double *d = (double *)malloc((size_t)(kk + 1) * sizeof(double));
    for (int i = 0; i < m; i++) {
        /* the kk smallest squared distances in ascending order (the head of the sorted list) */
        int nd = 0;
        for (int j = 0; j < m; j++) {
            const double v = d2_f64(p + 3 * idx[i], p + 3 * idx[j]);
            if (nd == kk && !(v < d[kk - 1])) continue;
            int q = nd < kk ? nd++ : kk - 1;
            while (q > 0 && v < d[q - 1]) {
                d[q] = d[q - 1];
                q--;
            }
            d[q] = v;
        }
        volatile double s = 0.0;
        for (int j = 0; j < kk; j++) s = s + sqrt(d[j]);  /* std::accumulate of sqrt'ed, ascending */
        avg[i] = s / (double)kk;
    }
    volatile double mean = 0.0;
    for (int i = 0; i < m; i++)
        if (avg[i] > 0) mean = mean + avg[i];
    mean = mean / (double)m;                          /* / valid_distances (= m) */
    volatile double sq = 0.0;
    for (int i = 0; i < m; i++) {
        volatile double t = avg[i] > 0 ? (avg[i] - mean) * (avg[i] - mean) : 0.0;
        sq = sq + t;
    }
    const double sd = sqrt(sq / (double)(m - 1));     /* Bessel */
    volatile double thr = std_ratio * sd;
    thr = mean + thr;
    int nk = 0;
    for (int i = 0; i < m; i++) {
        keep[i] = avg[i] > 0 && avg[i] < thr;
        nk += keep[i];
    }
    free(avg); free(d);
    return nk;
}

static int cmp_i32(const void *a, const void *b)
{
    const int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}

/* ---- one frame: turn_mask_to_point (:70-151) -----------------------------
 * scene: float32 [P,3] (construction.py:37 casts to float32); depth float32
 * [H,W]; seg uint8 [H,W] (aligned with depth); K = fx, fy, cx, cy; pose
 * row-major 4x4 (camera to world).
 * Outputs: kept masks in ascending id: labels[n], off[n+1] (CSR into pts),
 * pts = sorted unique scene ids (mask_info[id], :148).  stats[ST_NSTAT * c]
 * for every candidate id (c < 255), *n_cand of them.
 * Returns n >= 0; -1 if a depth pixel equals depth_trunc while the image has a
 * nonzero id (the reference's IndexError at :100); -2 if cap is too
 * small (*need = required). */
/* the frame's work; the neighbour ids go to a growable buffer *pb of *pcap entries */
static int s1_frame_core(int64_t P, const float *scene, int H, int W, const float *depth, const uint8_t *seg,
                         const double *K, const double *T, const orc_bp_params *prm, int32_t *labels, int64_t *off,
                         int32_t **pb, int64_t *pcap, int64_t *need, int32_t *stats, int32_t *n_cand)
{
    *need = 0;
    *n_cand = 0;
    off[0] = 0;
    for (int i = 0; i < 16; i++)
        if (isinf(T[i])) return 0;                    /* :73-74 */
    int present[256] = {0};
    int has_trunc = 0;
    for (int64_t i = 0; i < (int64_t)H * W; i++) {
        present[seg[i]] = 1;
        if ((double)depth[i] == prm->depth_trunc) has_trunc = 1;
    }
    int any_id = 0;
    for (int id = 1; id < 256; id++) any_id |= present[id];
    if (!any_id) return 0;                           /* :121-122 */
    if (has_trunc) return -1;

    double *mp = (double *)malloc((size_t)H * W * 3 * sizeof(double));
    double *vp = (double *)malloc((size_t)H * W * 3 * sizeof(double));
    int32_t *lab = (int32_t *)malloc((size_t)H * W * sizeof(int32_t));
    int32_t *sidx = (int32_t *)malloc((size_t)H * W * sizeof(int32_t));
    uint8_t *keep = (uint8_t *)malloc((size_t)H * W);
    float *q = (float *)malloc((size_t)H * W * 3 * sizeof(float));
    int32_t *cand = (int32_t *)malloc((size_t)(P + 1) * sizeof(int32_t));
    int32_t *nbr = NULL;  /* the ball query's accepted ids (then the frame's unique set) */
    int64_t nbr_cap = 0;
    int32_t *cnt = NULL;
    int ncnt_cap = 0;
    int n = 0;
    int64_t np = 0;
    const float r = (float)prm->ball_radius;
    const float r2 = r * r;

    for (int id = 1; id < 256; id++) {
        if (!present[id]) continue;
        int32_t *st = stats + ST_NSTAT * (*n_cand)++;
        memset(st, 0, ST_NSTAT * sizeof(int32_t));
        st[ST_ID] = id;
        /* (a2) mask points: seg == id among valid-depth pixels, row-major (:96-100) */
        int k = 0;
        for (int v = 0; v < H; v++)
            for (int u = 0; u < W; u++) {
                const int64_t i = (int64_t)v * W + u;
                const float d = depth[i];
                if (seg[i] != id || !(d > 0.0f) || !((double)d < prm->depth_trunc)) continue;
                world_point(K, T, u, v, d, mp + 3 * k);
                k++;
            }
        st[ST_NPIX] = k;
        if (k < prm->few_points) continue;           /* :101 */
        /* (a3) */
        const int nv = voxel_down(mp, k, prm->voxel_size, vp);
        st[ST_NVOX] = nv;
        /* (a4) denoise */
        dbscan(vp, nv, prm->dbscan_eps, prm->dbscan_min_points, lab);
        int maxl = -1;
        for (int i = 0; i < nv; i++)
            if (lab[i] > maxl) maxl = lab[i];
        if (maxl + 2 > ncnt_cap) {
            ncnt_cap = maxl + 2;
            cnt = (int32_t *)realloc(cnt, (size_t)ncnt_cap * sizeof(int32_t));
        }
        for (int c = 0; c < maxl + 2; c++) cnt[c] = 0;
        for (int i = 0; i < nv; i++) cnt[lab[i] + 1]++;  /* labels + 1, np.bincount */
        int m = 0;
        for (int i = 0; i < nv; i++)
            if (!((double)cnt[lab[i] + 1] < prm->component_min_fraction * (double)nv)) sidx[m++] = i;
        st[ST_NDB] = m;
        const int ns = statistical_outlier(vp, sidx, m, prm->sor_neighbors, prm->sor_std_ratio, keep);
        st[ST_NSOR] = ns;
        if (ns < prm->few_points) continue;          /* :109 */
        /* float32 mask points (:112) and the strict AABB crop (a5, :59-66) */
        int nq = 0;
        for (int i = 0; i < m; i++) {
            if (!keep[i]) continue;
            for (int c = 0; c < 3; c++) q[3 * nq + c] = (float)vp[3 * sidx[i] + c];
            nq++;
        }
        float lo[3], hi[3];
        for (int c = 0; c < 3; c++) {
            lo[c] = hi[c] = q[c];
            for (int i = 1; i < nq; i++) {
                if (q[3 * i + c] < lo[c]) lo[c] = q[3 * i + c];
                if (q[3 * i + c] > hi[c]) hi[c] = q[3 * i + c];
            }
        }
        int nc = 0;
        for (int64_t j = 0; j < P; j++) {
            const float *s = scene + 3 * j;
            if (s[0] > lo[0] && s[0] < hi[0] && s[1] > lo[1] && s[1] < hi[1] && s[2] > lo[2] && s[2] < hi[2])
                cand[nc++] = (int32_t)j;
        }
        st[ST_NCAND] = nc;
        /* (a6) ball_query K=20: the first K candidates in index order with d2 < r2 */
        if ((int64_t)nq * prm->ball_k > nbr_cap) {
            nbr_cap = (int64_t)nq * prm->ball_k;
            nbr = (int32_t *)realloc(nbr, (size_t)nbr_cap * sizeof(int32_t));
        }
        int64_t nn = 0;
        int covered = 0;
        for (int i = 0; i < nq; i++) {
            const float *qi = q + 3 * i;
            int c = 0;
            for (int t = 0; t < nc && c < prm->ball_k; t++) {
                const float *s = scene + 3 * (int64_t)cand[t];
                volatile float dx = qi[0] - s[0], dy = qi[1] - s[1], dz = qi[2] - s[2];
                volatile float xx = dx * dx;
                const float d2 = fmaf(dz, dz, fmaf(dy, dy, xx));
                if (d2 < r2) {
                    nbr[nn++] = cand[t];
                    c++;
                }
            }
            covered += c > 0;
        }
        st[ST_NCOV] = covered;
        /* (a7) coverage (:143-145) and the neighbour set (:141-142,148) */
        if ((double)covered / (double)nq < prm->coverage_threshold) continue;
        qsort(nbr, (size_t)nn, sizeof(int32_t), cmp_i32);
        int64_t u = 0;
        for (int64_t i = 0; i < nn; i++)
            if (u == 0 || nbr[i] != nbr[u - 1]) nbr[u++] = nbr[i];
        st[ST_NNBR] = (int32_t)u;
        st[ST_KEPT] = 1;
        if (np + u > *pcap) {
            while (np + u > *pcap) *pcap = 2 * *pcap + 1024;
            *pb = (int32_t *)realloc(*pb, (size_t)*pcap * sizeof(int32_t));
        }
        memcpy(*pb + np, nbr, (size_t)u * sizeof(int32_t));
        np += u;
        labels[n] = id;
        off[n + 1] = np;
        n++;
    }
    free(mp); free(vp); free(lab); free(sidx); free(keep); free(q); free(cand); free(nbr); free(cnt);
    *need = np;
    return n;
}

int orc_s1_frame(int64_t P, const float *scene, int H, int W, const float *depth, const uint8_t *seg,
                 const double *K, const double *T, const orc_bp_params *prm, int32_t *labels, int64_t *off,
                 int32_t *pts, int64_t cap, int64_t *need, int32_t *stats, int32_t *n_cand)
{
    int64_t bcap = 1 << 16;
    int32_t *buf = (int32_t *)malloc((size_t)bcap * sizeof(int32_t));
    const int n = s1_frame_core(P, scene, H, W, depth, seg, K, T, prm, labels, off, &buf, &bcap, need, stats, n_cand);
    if (n >= 0 && *need <= cap) memcpy(pts, buf, (size_t)*need * sizeof(int32_t));
    free(buf);
    if (n >= 0 && *need > cap) return -2;
    return n;
}

/* ---- many frames, OpenMP over frames (frames are independent, mask_backprojection.py:154-156;
 * the reference runs them one after another, construction.py:44-49) -------------------------
 * depth[f] / seg[f]: frame f's [H,W] arrays; K [F,4], T [F,16].  Per frame f: n_out[f] kept masks
 * (-1: the DEPTH_TRUNC error of :100), labels[256 f ..], off[257 f ..] (relative to the frame's
 * first id), stats[256 ST_NSTAT f ..], n_cand[f].  Returns a handle; *total = the frames' neighbour
 * ids, which orc_s1_batch_take copies out (frames in order) before freeing the handle. */
typedef struct {
    int F;
    int32_t **pts;
    int64_t *np;
} orc_s1_batch_t;

void *orc_s1_batch(int64_t P, const float *scene, int F, int H, int W, const float *const *depth,
                   const uint8_t *const *seg, const double *K, const double *T, const orc_bp_params *prm,
                   int nthreads, int32_t *n_out, int32_t *labels, int64_t *off, int32_t *stats, int32_t *n_cand,
                   int64_t *total)
{
    orc_s1_batch_t *h = (orc_s1_batch_t *)calloc(1, sizeof(orc_s1_batch_t));
    h->F = F;
    h->pts = (int32_t **)calloc((size_t)F + 1, sizeof(int32_t *));
    h->np = (int64_t *)calloc((size_t)F + 1, sizeof(int64_t));
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for (int f = 0; f < F; f++) {
        int64_t bcap = 1 << 16, need = 0;
        int32_t *buf = (int32_t *)malloc((size_t)bcap * sizeof(int32_t));
        const int n = s1_frame_core(P, scene, H, W, depth[f], seg[f], K + 4 * (size_t)f, T + 16 * (size_t)f, prm,
                                    labels + 256 * (size_t)f, off + 257 * (size_t)f, &buf, &bcap, &need,
                                    stats + (size_t)256 * ST_NSTAT * f, n_cand + f);
        n_out[f] = n;
        h->pts[f] = buf;
        h->np[f] = n >= 0 ? need : 0;
    }
    int64_t t = 0;
    for (int f = 0; f < F; f++) t += h->np[f];
    *total = t;
    return h;
}

void orc_s1_batch_take(void *hp, int32_t *pts)
{
    orc_s1_batch_t *h = (orc_s1_batch_t *)hp;
    int64_t o = 0;
    for (int f = 0; f < h->F; f++) {
        if (pts && h->np[f]) memcpy(pts + o, h->pts[f], (size_t)h->np[f] * sizeof(int32_t));
        o += h->np[f];
        free(h->pts[f]);
    }
    free(h->pts);
    free(h->np);
    free(h);
}
