// mc_pp_kernels.inl — post-processing of the clustered objects on gfx950.
//
// The reference's utils/post_process.py:173-195 per scene:
//   dbscan_process (:104-123)   Open3D DBSCAN(eps 0.1, min 4) of each node's points, one object per
//                               label class (class 0 = noise), in list(node.point_ids) order;
//   filter_point (:40-101)      per object point: frames of the node where it is seen (pfm) and where
//                               a mask of the node holds it; the detection-ratio filter; every node mask
//                               assigned to the object it intersects most (coverage = |m ∩ o| / |o|);
//   merge_overlapping_objects   greedy i < j pass over all kept objects with the bbox test
//   (:7-37)                     (utils/geometry.py:3-7) and the 0.8 intersection ratios.
//
// Layout: the nodes' points are one entry array (node k owns entries [pt_off[k], pt_off[k+1]) in
// its list order); every per-entry scratch array is indexed by entry, so nodes never share scratch.
// k_pp_dbscan and k_pp_filter are persistent workgroups taking nodes largest-first from a ticket.

namespace mc {

constexpr int kPPObjChunk = 1024;  // per-wave LDS counters of mask ∩ object
constexpr int kPPBoxChunk = 256;   // per-workgroup LDS bbox / kept-point accumulators
constexpr int kPPSlots = 16;       // objects per point in the intersection index (grown on demand)
constexpr int kPPLdsUF = 8192;     // nodes up to this many points keep their union-find in LDS

struct PPDev {
    double eps2, ce, thr, ratio;
    int minpts;
};

// order-preserving map of a double onto u64 (no NaNs on this path): min/max by integer atomics
__device__ __forceinline__ unsigned long long pp_ord(double v)
{
    const unsigned long long u = __double_as_longlong(v);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double pp_unord(unsigned long long u)
{
    return __longlong_as_double((u >> 63) ? (u & 0x7FFFFFFFFFFFFFFFull) : ~u);
}

__global__ __launch_bounds__(256) void k_pp_gather(const double *__restrict__ scene, const int *__restrict__ pts, int64_t E,
                                                   double *__restrict__ xyz)
{
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < 3 * E; i += gridDim.x * 256ll)
        xyz[i] = scene[3 * static_cast<int64_t>(pts[i / 3]) + i % 3];
}

// block min / max of 3 doubles over NT threads, broadcast; red holds 6 * NT/64 doubles
template <int NT>
__device__ __forceinline__ void pp_block_minmax3(double mn[3], double mx[3], double *red)
{
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const double lo = wave_min_d(mn[c]), hi = wave_max_d(mx[c]);
        if (lane == 0) {
            red[c * NW + wv] = lo;
            red[(3 + c) * NW + wv] = hi;
        }
    }
    sync_global();
#pragma unroll
    for (int c = 0; c < 3; c++) {
        mn[c] = red[c * NW];
        mx[c] = red[(3 + c) * NW];
        for (int w = 1; w < NW; w++) {
            mn[c] = fmin(mn[c], red[c * NW + w]);
            mx[c] = fmax(mx[c], red[(3 + c) * NW + w]);
        }
    }
    sync_global();
}

// DBSCAN of every node (utils/post_process.py:109): labels -> object index within the node
// (class order: noise first when present, then clusters by smallest core point), object sizes.
// the 27 cells around (cx, cy, cz) over the bucket-ordered copies (key, xyz, index): the loads of
// one bucket are independent of each other, not a cell -> point -> coordinate chain
template <typename Fn>
__device__ __forceinline__ void pp_walk27(const BpCells &g, const unsigned long long *__restrict__ sk,
                                          const double *__restrict__ sx, const int *__restrict__ si, int cx, int cy,
                                          int cz, Fn &&fn)
{
    for (int z = cz - 1; z <= cz + 1; z++)
        for (int y = cy - 1; y <= cy + 1; y++)
            for (int x = cx - 1; x <= cx + 1; x++) {
                if (x < 0 || y < 0 || z < 0 || x > g.cmax[0] || y > g.cmax[1] || z > g.cmax[2]) continue;
                const unsigned long long key = pack3(x, y, z);
                const unsigned bk = mod_mul(bp_hash3(x, y, z), g.nb);
                const int k1 = g.bs[bk + 1];
                for (int q = g.bs[bk]; q < k1; q++)
                    if (sk[q] == key) fn(si[q], sx + 3 * static_cast<int64_t>(q));
            }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_pp_dbscan(
    int N, const int *__restrict__ order, int *__restrict__ ticket, const int64_t *__restrict__ pt_off, PPDev pr,
    const double *__restrict__ xyz, unsigned long long *__restrict__ pcell, int *__restrict__ pbkt,
    int *__restrict__ bcnt, int *__restrict__ bstart, int *__restrict__ blist, int *__restrict__ ncnt,
    int *__restrict__ par, int *__restrict__ root, int *__restrict__ rnk, int *__restrict__ lab,
    int *__restrict__ ccnt, int *__restrict__ nob, int *__restrict__ nsh, unsigned long long *__restrict__ skey,
    double *__restrict__ sxyz, int *__restrict__ sidx)
{
    __shared__ double red[6 * (NT / 64)];
    __shared__ int ws[NT / 64];
    __shared__ int s_k;
    __shared__ int s_par[kPPLdsUF];  // union-find in LDS when the node fits: global-memory find chains
                                     // (a dependent load per step) made the unions the whole cost
    const int t = threadIdx.x;
    while (true) {
        if (t == 0) s_k = atomicAdd(ticket, 1);
        sync_global();
        const int kk = s_k;
        sync_global();
        if (kk >= N) break;
        const int k = order[kk];
        const int64_t e0 = pt_off[k];
        const int n = static_cast<int>(pt_off[k + 1] - e0);
        const double *P = xyz + 3 * e0;
        unsigned long long *pc = pcell + e0;
        int *pb = pbkt + e0, *bc = bcnt + 2 * e0 + k, *bs = bstart + 2 * e0 + k, *bl = blist + e0;
        int *nc = ncnt + e0, *pa = par + e0, *ro = root + e0, *rk = rnk + e0, *lb = lab + e0, *cc = ccnt + e0 + k;
        const unsigned nb = 2u * static_cast<unsigned>(n);
        // 1. bounding box -> grid origin (cells of 1.01 eps: every eps-neighbour is in the 27 cells)
        double mn[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, mx[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
        for (int i = t; i < n; i += NT)
#pragma unroll
            for (int c = 0; c < 3; c++) {
                mn[c] = fmin(mn[c], P[3 * i + c]);
                mx[c] = fmax(mx[c], P[3 * i + c]);
            }
        pp_block_minmax3<NT>(mn, mx, red);
        BpCells g;
        g.pc = pc;
        g.bs = bs;
        g.bl = bl;
        g.nb = nb;
#pragma unroll
        for (int c = 0; c < 3; c++) g.cmax[c] = static_cast<int>(floor((mx[c] - mn[c]) / pr.ce));
        // 2. cells + bucket counts (bucket counters are zero at rest)
        for (int i = t; i < n; i += NT) {
            int cxyz[3];
#pragma unroll
            for (int c = 0; c < 3; c++) cxyz[c] = static_cast<int>(floor((P[3 * i + c] - mn[c]) / pr.ce));
            pc[i] = pack3(cxyz[0], cxyz[1], cxyz[2]);
            const unsigned b = mod_mul(bp_hash3(cxyz[0], cxyz[1], cxyz[2]), nb);
            pb[i] = static_cast<int>(b);
            atomicAdd(&bc[b], 1);
        }
        for (int i = t; i <= n; i += NT) cc[i] = 0;
        sync_global();
        // 3. bucket starts
        {
            int carry = 0;
            for (int b0 = 0; b0 < static_cast<int>(nb); b0 += NT) {
                const int b = b0 + t;
                const int v = b < static_cast<int>(nb) ? ld_agent(&bc[b]) : 0;
                int tot;
                const int ex = block_excl_scan<NT>(v, ws, tot);
                if (b < static_cast<int>(nb)) bs[b] = carry + ex;
                carry += tot;
            }
            if (t == 0) bs[nb] = carry;
        }
        sync_global();
        // 4. counting-sort scatter (bucket counters return to zero)
        unsigned long long *sk = skey + e0;
        double *sx = sxyz + 3 * e0;
        int *si = sidx + e0;
        for (int i = t; i < n; i += NT) {
            const int b = pb[i];
            const int q = bs[b] + atomicSub(&bc[b], 1) - 1;
            bl[q] = i;
            sk[q] = pc[i];
            si[q] = i;
#pragma unroll
            for (int c = 0; c < 3; c++) sx[3 * q + c] = P[3 * i + c];
        }
        sync_global();
        auto cell_of = [&](int i, int &x, int &y, int &z) { unpack3(pc[i], x, y, z); };
        // 5. eps-neighbour counts, self included (nanoflann radius search: d2 < eps^2)
        for (int i = t; i < n; i += NT) {
            int x, y, z;
            cell_of(i, x, y, z);
            int cnt = 0;
            const double *pi = P + 3 * i;
            pp_walk27(g, sk, sx, si, x, y, z, [&](int, const double *pj) { cnt += bp_d2(pi, pj) < pr.eps2 ? 1 : 0; });
            nc[i] = cnt;
            if (n <= kPPLdsUF) s_par[i] = i;
            else pa[i] = i;
        }
        sync_global();
        // 6. core points connected within eps: union-find, root = smallest index
        for (int i = t; i < n; i += NT) {
            if (nc[i] < pr.minpts) continue;
            int x, y, z;
            cell_of(i, x, y, z);
            const double *pi = P + 3 * i;
            pp_walk27(g, sk, sx, si, x, y, z, [&](int j, const double *pj) {
                if (j < i && nc[j] >= pr.minpts && bp_d2(pi, pj) < pr.eps2) {
                    if (n <= kPPLdsUF) uf_unite_s(s_par, i, j);
                    else uf_unite(pa, i, j);
                }
            });
        }
        sync_global();
        // 7. clusters numbered by their smallest core point (Open3D seeds in index order)
        int ncl;
        {
            int carry = 0;
            for (int i0 = 0; i0 < n; i0 += NT) {
                const int i = i0 + t;
                int isr = 0;
                if (i < n && nc[i] >= pr.minpts) {
                    const int r = n <= kPPLdsUF ? uf_find_s(s_par, i) : uf_find(pa, i);
                    ro[i] = r;
                    isr = r == i ? 1 : 0;
                }
                int tot;
                const int ex = block_excl_scan<NT>(isr, ws, tot);
                if (isr) rk[i] = carry + ex;
                carry += tot;
            }
            ncl = carry;
        }
        sync_global();
        // 8. labels: a border point joins the first cluster that reaches it = the adjacent cluster
        //    of smallest number; class = label + 1 (post_process.py:109)
        for (int i = t; i < n; i += NT) {
            int l;
            if (nc[i] >= pr.minpts) {
                l = rk[ro[i]];
            } else {
                int x, y, z;
                cell_of(i, x, y, z);
                const double *pi = P + 3 * i;
                int mr = INT_MAX;
                pp_walk27(g, sk, sx, si, x, y, z, [&](int j, const double *pj) {
                    if (nc[j] >= pr.minpts && bp_d2(pi, pj) < pr.eps2) mr = min(mr, ro[j]);
                });
                l = mr == INT_MAX ? -1 : rk[mr];
            }
            lb[i] = l + 1;
            atomicAdd(&cc[l + 1], 1);
        }
        sync_global();
        // 9. objects = non-empty classes (:115-118): the noise class only when it is non-empty;
        //    object = class - shift
        if (t == 0) {
            const int noise = ld_agent(&cc[0]) > 0 ? 1 : 0;
            nob[k] = ncl + noise;
            nsh[k] = 1 - noise;
        }
        sync_global();
    }
}

// Large nodes (more than a threshold of points, e.g. a floor of ScanNet++ size) are split over
// many workgroups: the grid of a node is built by one workgroup (k_pp_big_grid), the neighbour
// counts and the core-point unions run on (node, 512-point chunk) items over the whole chip
// (k_pp_big_walk), and ranks / labels / objects again per node (k_pp_big_label).  Same steps and
// results as k_pp_dbscan.
struct PPBig {
    const int64_t *pt_off;
    const double *xyz;
    unsigned long long *pcell;
    int *pbkt, *bcnt, *bstart, *blist, *ncnt, *par, *root, *rnk, *lab, *ccnt;
    int *gcm;  // per node: cmax[3]
};

__device__ __forceinline__ BpCells pp_cells(const PPBig &b, int k, int64_t e0, int n)
{
    BpCells g;
    g.pc = b.pcell + e0;
    g.bs = b.bstart + 2 * e0 + k;
    g.bl = b.blist + e0;
    g.nb = 2u * static_cast<unsigned>(n);
#pragma unroll
    for (int c = 0; c < 3; c++) g.cmax[c] = b.gcm[3 * k + c];
    return g;
}

template <int NT>
__global__ __launch_bounds__(NT) void k_pp_big_grid(int nbig, const int *__restrict__ big, PPDev pr, PPBig b)
{
    __shared__ double red[6 * (NT / 64)];
    __shared__ int ws[NT / 64];
    const int t = threadIdx.x;
    for (int q = blockIdx.x; q < nbig; q += gridDim.x) {
        const int k = big[q];
        const int64_t e0 = b.pt_off[k];
        const int n = static_cast<int>(b.pt_off[k + 1] - e0);
        const double *P = b.xyz + 3 * e0;
        unsigned long long *pc = b.pcell + e0;
        int *pb = b.pbkt + e0, *bc = b.bcnt + 2 * e0 + k, *bs = b.bstart + 2 * e0 + k, *bl = b.blist + e0;
        int *pa = b.par + e0, *cc = b.ccnt + e0 + k;
        const unsigned nb = 2u * static_cast<unsigned>(n);
        double mn[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, mx[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
        for (int i = t; i < n; i += NT)
#pragma unroll
            for (int c = 0; c < 3; c++) {
                mn[c] = fmin(mn[c], P[3 * i + c]);
                mx[c] = fmax(mx[c], P[3 * i + c]);
            }
        pp_block_minmax3<NT>(mn, mx, red);
        if (t == 0)
#pragma unroll
            for (int c = 0; c < 3; c++) b.gcm[3 * k + c] = static_cast<int>(floor((mx[c] - mn[c]) / pr.ce));
        for (int i = t; i < n; i += NT) {
            int cxyz[3];
#pragma unroll
            for (int c = 0; c < 3; c++) cxyz[c] = static_cast<int>(floor((P[3 * i + c] - mn[c]) / pr.ce));
            pc[i] = pack3(cxyz[0], cxyz[1], cxyz[2]);
            const unsigned h = mod_mul(bp_hash3(cxyz[0], cxyz[1], cxyz[2]), nb);
            pb[i] = static_cast<int>(h);
            atomicAdd(&bc[h], 1);
            pa[i] = i;
        }
        for (int i = t; i <= n; i += NT) cc[i] = 0;
        sync_global();
        int carry = 0;
        for (int b0 = 0; b0 < static_cast<int>(nb); b0 += NT) {
            const int h = b0 + t;
            const int v = h < static_cast<int>(nb) ? ld_agent(&bc[h]) : 0;
            int tot;
            const int ex = block_excl_scan<NT>(v, ws, tot);
            if (h < static_cast<int>(nb)) bs[h] = carry + ex;
            carry += tot;
        }
        if (t == 0) bs[nb] = carry;
        sync_global();
        for (int i = t; i < n; i += NT) {
            const int h = pb[i];
            bl[bs[h] + atomicSub(&bc[h], 1) - 1] = i;
        }
        sync_global();
    }
}

// PASS 0: eps-neighbour counts; PASS 1: unions of core points (root = smallest index)
template <int NT, int PASS>
__global__ __launch_bounds__(NT) void k_pp_big_walk(int nitems, const int2 *__restrict__ items, PPDev pr, PPBig b)
{
    for (int q = blockIdx.x; q < nitems; q += gridDim.x) {
        const int k = items[q].x;
        const int64_t e0 = b.pt_off[k];
        const int n = static_cast<int>(b.pt_off[k + 1] - e0);
        const int i = items[q].y + static_cast<int>(threadIdx.x);
        if (i >= n) continue;
        const BpCells g = pp_cells(b, k, e0, n);
        const double *P = b.xyz + 3 * e0;
        int *nc = b.ncnt + e0;
        int x, y, z;
        unpack3(g.pc[i], x, y, z);
        const double *pi = P + 3 * i;
        if (PASS == 0) {
            int cnt = 0;
            for (int R = 0; R <= 1; R++)
                bp_shell(g, x, y, z, R, [&](int j) { cnt += bp_d2(pi, P + 3 * j) < pr.eps2 ? 1 : 0; });
            nc[i] = cnt;
        } else {
            if (nc[i] < pr.minpts) continue;
            int *pa = b.par + e0;
            for (int R = 0; R <= 1; R++)
                bp_shell(g, x, y, z, R, [&](int j) {
                    if (j < i && nc[j] >= pr.minpts && bp_d2(pi, P + 3 * j) < pr.eps2) uf_unite(pa, i, j);
                });
        }
    }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_pp_big_label(int nbig, const int *__restrict__ big, PPDev pr, PPBig b,
                                                     int *__restrict__ nob, int *__restrict__ nsh)
{
    __shared__ int ws[NT / 64];
    const int t = threadIdx.x;
    for (int q = blockIdx.x; q < nbig; q += gridDim.x) {
        const int k = big[q];
        const int64_t e0 = b.pt_off[k];
        const int n = static_cast<int>(b.pt_off[k + 1] - e0);
        const BpCells g = pp_cells(b, k, e0, n);
        const double *P = b.xyz + 3 * e0;
        int *nc = b.ncnt + e0, *pa = b.par + e0, *ro = b.root + e0, *rk = b.rnk + e0, *lb = b.lab + e0;
        int *cc = b.ccnt + e0 + k;
        int carry = 0;
        for (int i0 = 0; i0 < n; i0 += NT) {
            const int i = i0 + t;
            int isr = 0;
            if (i < n && nc[i] >= pr.minpts) {
                const int r = uf_find(pa, i);
                ro[i] = r;
                isr = r == i ? 1 : 0;
            }
            int tot;
            const int ex = block_excl_scan<NT>(isr, ws, tot);
            if (isr) rk[i] = carry + ex;
            carry += tot;
        }
        const int ncl = carry;
        sync_global();
        for (int i = t; i < n; i += NT) {
            int l;
            if (nc[i] >= pr.minpts) {
                l = rk[ro[i]];
            } else {
                int x, y, z;
                unpack3(g.pc[i], x, y, z);
                const double *pi = P + 3 * i;
                int mr = INT_MAX;
                for (int R = 0; R <= 1; R++)
                    bp_shell(g, x, y, z, R, [&](int j) {
                        if (nc[j] >= pr.minpts && bp_d2(pi, P + 3 * j) < pr.eps2) mr = min(mr, ro[j]);
                    });
                l = mr == INT_MAX ? -1 : rk[mr];
            }
            lb[i] = l + 1;
            atomicAdd(&cc[l + 1], 1);
        }
        sync_global();
        if (t == 0) {
            const int noise = ld_agent(&cc[0]) > 0 ? 1 : 0;
            nob[k] = ncl + noise;
            nsh[k] = 1 - noise;
        }
        sync_global();
    }
}

// wave-wide first maximum (value, index): larger value wins, smaller index on ties
__device__ __forceinline__ void pp_wave_argmax(int &v, int &ix)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const int ov = __shfl_xor(v, d, 64), oi = __shfl_xor(ix, d, 64);
        if (ov > v || (ov == v && oi < ix)) {
            v = ov;
            ix = oi;
        }
    }
}

// filter_point (post_process.py:40-101) of every node; posmap = one P-entry map per workgroup,
// -1 at rest.
__global__ __launch_bounds__(256) void k_pp_filter(
    int N, const int *__restrict__ order, int *__restrict__ ticket, PPDev pr, int FW, int64_t P,
    const int64_t *__restrict__ pt_off, const int *__restrict__ pts, const unsigned long long *__restrict__ nvf,
    const int64_t *__restrict__ hit_off, const int64_t *__restrict__ qoff, const int *__restrict__ qmask,
    const int *__restrict__ qfpos, const int64_t *__restrict__ mask_off, const int *__restrict__ mask_pts,
    const unsigned long long *__restrict__ pfm, const double *__restrict__ xyz, const int *__restrict__ lab,
    const int *__restrict__ ccnt, const int *__restrict__ nob, const int *__restrict__ nsh,
    const int *__restrict__ obj_base,
    int *__restrict__ posmap, unsigned long long *__restrict__ hit, int *__restrict__ cvid,
    int *__restrict__ qobj, double *__restrict__ qcov, int *__restrict__ obj_nmask, int *__restrict__ obj_nvalid,
    double *__restrict__ obj_box, int *__restrict__ ent_obj)
{
    __shared__ int s_cnt[4][kPPObjChunk];
    __shared__ unsigned long long s_box[kPPBoxChunk * 6];
    __shared__ int s_nv[kPPBoxChunk];
    __shared__ int s_k;
    const int t = threadIdx.x, lane = lane_id(), wv = t >> 6;
    int *pm = posmap + static_cast<int64_t>(blockIdx.x) * P;
    while (true) {
        if (t == 0) s_k = atomicAdd(ticket, 1);
        sync_global();
        const int kk = s_k;
        sync_global();
        if (kk >= N) break;
        const int k = order[kk];
        const int64_t e0 = pt_off[k];
        const int n = static_cast<int>(pt_off[k + 1] - e0);
        const int no = nob[k], sh = nsh[k], ob = obj_base[k];
        const int *lb = lab + e0, *cc = ccnt + e0 + k;
        const int W = n ? static_cast<int>((hit_off[k + 1] - hit_off[k]) / n) : 0;
        unsigned long long *hk = hit + hit_off[k];
        const unsigned long long *vf = nvf + static_cast<int64_t>(k) * FW;
        // 1. position map; frames of the node's visible frames the point is seen in (:45-58)
        for (int i = t; i < n; i += 256) {
            const int p = pts[e0 + i];
            pm[p] = i;
            int c = 0;
            for (int w = 0; w < FW; w++) c += __popcll(pfm[static_cast<int64_t>(p) * FW + w] & vf[w]);
            cvid[e0 + i] = c;
        }
        sync_global();
        // 2. masks of the node, a wave each (:68-81): frame bits of the points they hold, and the
        //    object of largest intersection
        const int64_t q0 = qoff[k], q1 = qoff[k + 1];
        for (int64_t q = q0 + wv; q < q1; q += 4) {
            const int m = qmask[q], fp = qfpos[q];
            const int64_t a = mask_off[m], b = mask_off[m + 1];
            int best = -1, largest = 0;
            for (int c0 = 0; c0 < no; c0 += kPPObjChunk) {
                const int cn = min(kPPObjChunk, no - c0);
                for (int c = lane; c < cn; c += 64) s_cnt[wv][c] = 0;
                __builtin_amdgcn_wave_barrier();
                for (int64_t j = a + lane; j < b; j += 64) {
                    const int li = pm[mask_pts[j]];
                    if (li < 0) continue;
                    if (c0 == 0) atomicOr(&hk[static_cast<int64_t>(li) * W + (fp >> 6)], 1ull << (fp & 63));
                    const int o = lb[li] - sh - c0;
                    if (o >= 0 && o < cn) atomicAdd(&s_cnt[wv][o], 1);
                }
                __builtin_amdgcn_wave_barrier();
                int v = 0, ix = INT_MAX;
                for (int c = lane; c < cn; c += 64) {
                    const int x = s_cnt[wv][c];
                    if (x > v) {
                        v = x;
                        ix = c;
                    }
                }
                pp_wave_argmax(v, ix);
                if (v > largest) {
                    largest = v;
                    best = c0 + ix;
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (lane == 0) {
                qobj[q] = best >= 0 ? ob + best : -1;
                qcov[q] = best >= 0 ? static_cast<double>(largest) / static_cast<double>(cc[best + sh]) : 0.0;
                if (best >= 0) atomicAdd(&obj_nmask[ob + best], 1);
            }
        }
        sync_global();
        // 3. detection ratio (:93-95), kept-point counts and bboxes of all object points (:99)
        for (int c0 = 0; c0 < no; c0 += kPPBoxChunk) {
            const int cn = min(kPPBoxChunk, no - c0);
            for (int c = t; c < cn; c += 256) {
                s_nv[c] = 0;
#pragma unroll
                for (int d = 0; d < 3; d++) {
                    s_box[6 * c + d] = ~0ull;
                    s_box[6 * c + 3 + d] = 0ull;
                }
            }
            sync_global();
            for (int i = t; i < n; i += 256) {
                const int o = lb[i] - sh;
                int cnode = 0;
                for (int w = 0; w < W; w++)
                    cnode += __popcll(__hip_atomic_load(&hk[static_cast<int64_t>(i) * W + w], __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT));
                const bool valid = static_cast<double>(cnode) / (static_cast<double>(cvid[e0 + i]) + 1e-6) > pr.thr;
                if (c0 == 0) ent_obj[e0 + i] = valid ? ob + o : -1;
                if (o - c0 < 0 || o - c0 >= cn) continue;
                const int oc = o - c0;
                if (valid) atomicAdd(&s_nv[oc], 1);
#pragma unroll
                for (int d = 0; d < 3; d++) {
                    const unsigned long long u = pp_ord(xyz[3 * (e0 + i) + d]);
                    atomicMin(&s_box[6 * oc + d], u);
                    atomicMax(&s_box[6 * oc + 3 + d], u);
                }
            }
            sync_global();
            for (int c = t; c < cn; c += 256) {
                obj_nvalid[ob + c0 + c] = s_nv[c];
#pragma unroll
                for (int d = 0; d < 6; d++) obj_box[6 * static_cast<int64_t>(ob + c0 + c) + d] = pp_unord(s_box[6 * c + d]);
            }
            sync_global();
        }
        // 4. the position map returns to -1
        for (int i = t; i < n; i += 256) pm[pts[e0 + i]] = -1;
        sync_global();
    }
}

// intersection index: the kept objects holding each point (fixed slots; overflow -> regrow)
__global__ __launch_bounds__(256) void k_pp_index(int64_t E, const int *__restrict__ pts, const int *__restrict__ ent_obj,
                                                  const int *__restrict__ kidx, int slots, int *__restrict__ pcnt,
                                                  int *__restrict__ plist, int *__restrict__ maxcnt)
{
    for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < E; e += gridDim.x * 256ll) {
        const int o = ent_obj[e];
        if (o < 0) continue;
        const int kk = kidx[o];
        if (kk < 0) continue;
        const int p = pts[e];
        const int s = atomicAdd(&pcnt[p], 1);
        if (s < slots) plist[static_cast<int64_t>(p) * slots + s] = kk;
        atomicMax(maxcnt, s + 1);
    }
}

// |set_i ∩ set_j| for every pair of kept objects sharing a point (dense K x K, i < j)
__global__ __launch_bounds__(256) void k_pp_pairs(int64_t P, int slots, const int *__restrict__ pcnt,
                                                  const int *__restrict__ plist, int K, int *__restrict__ inter)
{
    for (int64_t p = blockIdx.x * 256ll + threadIdx.x; p < P; p += gridDim.x * 256ll) {
        const int c = pcnt[p];
        if (c < 2) continue;
        const int *l = plist + p * slots;
        for (int a = 0; a < c; a++)
            for (int b = a + 1; b < c; b++) {
                const int x = min(l[a], l[b]), y = max(l[a], l[b]);
                atomicAdd(&inter[static_cast<int64_t>(x) * K + y], 1);
            }
    }
}

// decision of every pair i < j (post_process.py:24-29): 1 = i merged away, 2 = j merged away
// The non-zero decisions are also appended to a list (order-free; capacity cap) so that the host
// can run the greedy pass over them alone when they fit.
__global__ __launch_bounds__(256) void k_pp_decide(int K, PPDev pr, const double *__restrict__ box,
                                                   const int *__restrict__ len, const int *__restrict__ inter,
                                                   unsigned char *__restrict__ dec, int cap, int *__restrict__ nlist,
                                                   int2 *__restrict__ list)
{
    const int64_t tot = static_cast<int64_t>(K) * K;
    for (int64_t x = blockIdx.x * 256ll + threadIdx.x; x < tot; x += gridDim.x * 256ll) {
        const int i = static_cast<int>(x / K), j = static_cast<int>(x % K);
        if (j <= i) continue;
        const double *bi = box + 6 * static_cast<int64_t>(i), *bj = box + 6 * static_cast<int64_t>(j);
        bool ov = true;
#pragma unroll
        for (int d = 0; d < 3; d++)
            if (bi[d] > bj[3 + d] || bj[d] > bi[3 + d]) ov = false;  // utils/geometry.py:3-7
        unsigned char r = 0;
        if (ov) {
            const double in = static_cast<double>(inter[x]);
            if (in / static_cast<double>(len[i]) > pr.ratio) r = 1;
            else if (in / static_cast<double>(len[j]) > pr.ratio) r = 2;
        }
        dec[x] = r;
        if (r) {
            const int at = atomicAdd(nlist, 1);
            if (at < cap) list[at] = make_int2(i, r == 1 ? -1 - j : j);
        }
    }
}

// the greedy pass (post_process.py:14-29): sequential in i, every j of one i in parallel
__global__ __launch_bounds__(1024) void k_pp_greedy(int K, const unsigned char *__restrict__ dec,
                                                    unsigned char *__restrict__ inv)
{
    __shared__ int s_flag;
    const int t = threadIdx.x;
    for (int i = t; i < K; i += 1024) inv[i] = 0;
    sync_global();
    for (int i = 0; i < K; i++) {
        if (t == 0) s_flag = 0;
        sync_global();
        if (inv[i]) continue;  // uniform: written before the last barrier
        const unsigned char *d = dec + static_cast<int64_t>(i) * K;
        int f = 0;
        for (int j = i + 1 + t; j < K; j += 1024) {
            if (inv[j]) continue;
            const unsigned char r = d[j];
            if (r == 1) f = 1;
            else if (r == 2) inv[j] = 1;
        }
        if (f) s_flag = 1;
        sync_global();
        if (t == 0 && s_flag) inv[i] = 1;
        sync_global();
    }
}

}  // namespace mc
