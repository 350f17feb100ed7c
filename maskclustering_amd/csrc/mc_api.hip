// mc_api.hip — C-ABI of libmcgraph: context, scene upload, S2–S6 orchestration, getters.
// Single translation unit: the kernels live in mc_kernels.inl.
#include <dlfcn.h>
#include <rccl/rccl.h>  // types only: the library loads RCCL at mc_ctx_attach_comm / mc_ctx_comm_init (dlopen)

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
#include <vector>

#include "mc_internal.hpp"
#include "mc_kernels.inl"
#include "mc_bp_kernels.inl"
#include "mc_pp_kernels.inl"
#include "mc_eval_kernels.inl"
#include "mc_io_kernels.inl"
#include "mc_shard_kernels.inl"
#include "mc_ov_kernels.inl"
#include "mc_setorder.inl"

using mc::DevBuf;
using mc::McError;
using mc::TimedScope;
using mc::ceil_div;

namespace {

// device-side statistics block (copied to pinned host memory in one transfer)
enum Stat : int {
    ST_NBND = 0,      // boundary points
    ST_NNZC = 1,      // contained entries after undo
    ST_N0 = 2,        // level-0 nodes
    ST_NTHR = 3,      // thresholds
    ST_THR_STATUS = 4,
    ST_K = 5,         // final objects
    ST_WORDS = 6,     // point-bitmap words
    ST_NPTS = 7,      // object points (sum)
    ST_OBJOVF = 8,    // a point in more objects than the per-point fast path holds
    ST_COUNT = 9,
};

// S6 levels t >= 1 of scenes with at most this many level-0 nodes run the component labelling in
// one workgroup (k6_components, one launch); level 0 and larger scenes use the multi-workgroup
// kernels (k6_compress .. k6_memscatter, five launches)
constexpr int kFusedComponentsMaxN0 = 32768;

}  // namespace

struct mc_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    hipStream_t side = nullptr;                 // S3: workgroup-per-mask kernel beside the wave kernel
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipStream_t cls_stream[mc::kBpStreamClasses] = {};  // S1 denoise: the LDS size classes run side by side
    hipEvent_t ev_cls[mc::kBpStreamClasses] = {};
    std::string err;
    mc::KernelTimer timer;
    int *h_stats = nullptr;  // pinned
    int *h_bppack = nullptr;   // pinned per-batch S1 readback (k_bp_pack), h_bppack_n ints
    int *h_bpstat = nullptr;   // pinned per-batch statistics block
    hipEvent_t ev_pack = nullptr;  // the last batch's h_bppack copy (unpacked under the next batch)
    size_t h_bppack_n = 0;
    // pinned staging ring of mc_backproject_frames (two chunks, ping-pong)
    char *h_stage[2] = {nullptr, nullptr};
    size_t stage_bytes = 0;
    hipEvent_t ev_stage[2] = {};
    bool stage_used[2] = {false, false};
    // host frames staged batch by batch on their own stream while the previous batch computes
    hipStream_t copy = nullptr;
    hipEvent_t ev_up = nullptr;
    struct BpUpload *bp_up = nullptr;  // set for the duration of mc_backproject_frames' S1 call

    // ---- scene ----
    bool have_scene = false, have_graph = false, have_nodes = false, have_cluster = false;
    bool nodes_from_graph = false;
    int64_t P = 0;
    int F = 0, FW = 0, M = 0, M_in = 0;
    int nnz = 0;
    std::vector<int32_t> h_col, h_label, h_in_index, h_off;
    DevBuf d_mask_off, d_mask_pts, d_mask_col, d_mask_label, d_frame_start, d_valid;
    // ---- S2 ----
    DevBuf d_deg, d_pt_off, d_pt_list, d_boundary, d_pfm, d_scan_tmp;
    // ---- S3/S5 ----
    DevBuf d_ctmp, d_crow_len, d_useg, d_keep_cnt, d_node_flag, d_node_pos, d_c_off, d_c_idx, d_vf;
    // ---- S4 ----
    DevBuf d_hist, d_thr, d_isint, d_stats, d_s4rng;
    // ---- level-0 nodes ----
    int N0 = 0;        // host copy (valid after sync_stats or mc_nodes_set)
    int Mn = 0;        // mask-id space of C rows
    int64_t n0_pts_total = 0;
    DevBuf d_node0_g, d_n0_off, d_n0_len, d_n0_ptoff, d_n0_ptlen, d_n0_vf, d_user_cidx, d_user_pts;
    DevBuf d_owner0, d_node_of_mask, d_obj_of_mask, d_s3_small, d_s3_big, d_collen;
    int n_s3_small = 0, n_s3_big = 0;
    const int *n0_pool = nullptr;
    const int *n0_pts = nullptr;
    int64_t nnzC0 = 0;
    // ---- S6 ----
    DevBuf d_parent, d_root, d_isroot, d_rank, d_label, d_levels, d_memcnt, d_memoff, d_ublen, d_newoff;
    DevBuf d_members, d_colcnt, d_coloff, d_colnodes, d_ovf_n, d_scratch, d_touched, d_edges;
    DevBuf d_spread;  // spread slots of the S2 boundary counter
    DevBuf d_Nlev, d_final_label;
    DevBuf d_poolA, d_poolB, d_offA, d_offB, d_lenA, d_lenB, d_vfA, d_vfB, d_ownA, d_ownB, d_cap;
    DevBuf d_pmin, d_pmax, d_nwords, d_woff, d_bm, d_ptcnt, d_ptoff_out, d_pts_out;
    int scratch_n0 = -1;
    int n_iter = 0;
    // final object state (device pointers into the pools)
    const int *fin_off = nullptr, *fin_len = nullptr, *fin_pool = nullptr;
    const unsigned long long *fin_vf = nullptr;
    int K = 0;
    int64_t npts = 0;

    // ---- S1 back-projection ----
    int64_t P_scene = 0;
    bool have_points = false, have_bp = false;
    float grid_radius = -1.f;  // scene grid built for this ball radius
    unsigned gnb = 0;
    DevBuf d_scene, d_gcnt, d_gstart, d_gbkt, d_gcellk, d_gpts, d_gidx, d_gcell, d_gscan_tmp;
    DevBuf d_in_depth, d_in_seg, d_in_intr, d_in_pose, d_in_raw;
    DevBuf d_band, d_present, d_fflags, d_cand, d_npix, d_csidx, d_poff, d_slot_of, d_bpstat;
    DevBuf d_bpvid;  // per-batch valid-id map (k_bp_count -> k_bp_compact), 1 byte per pixel
    DevBuf d_slot_frame, d_slot_id, d_slot_np, d_slot_pix, d_slot_nv, d_slot_m, d_slot_ns, d_slot_box, d_slot_nn,
        d_slot_toff, d_slot_cov;
    DevBuf d_pix_list, d_hkey, d_hvid, d_hfirst, d_vox_entry, d_acc, d_vpts, d_pcell, d_pbkt, d_bcnt, d_bstart,
        d_blist, d_ncnt, d_par, d_droot, d_rnk, d_lab, d_ccnt, d_ssidx, d_avg, d_qpts;
    DevBuf d_bpbm, d_tmp, d_kflag, d_ksize, d_midx, d_moff, d_out_col, d_out_label, d_out_off, d_out_pts, d_bp_pts;
    DevBuf d_cls_list, d_nbl, d_lean, d_vox_order;  // denoise size-class slot lists; per-workgroup eps-neighbour lists, lean scratch
    // voxel_down_sample: per-pixel voxel ids and voxel lists of k_bp_voxel_lds; its overflow slots
    DevBuf d_vx_pvid, d_vx_list, d_vx_fb, d_bppack;
    DevBuf d_scanm;  // block sums of the per-batch multi-workgroup scans
    DevBuf d_slot_grid;  // denoise: grid origin / extent of the slots with points queued for the k-NN ring search
    int num_cu = 256;
    int64_t mem_budget = 0;  // bytes the S1 per-batch arrays may take (0: the default share, mc_backproject)
    size_t bp_px_cap = 0;  // mask-pixel capacity of the per-batch arrays (pixel-list positions)
    int bp_last_fb = 0;    // frames per batch at the end of the last mc_backproject
    bool bp_mfrac_obs = false;  // bp_mfrac comes from an earlier call's batches (not the initial guess)
    int64_t bp_redo = 0;   // batches redone after a mask-pixel overflow (all calls)
    int bp_f_cap = 0;      // frame capacity of the per-batch arrays
    size_t bp_fpx_cap = 0; // frame-pixel capacity (the valid-id map)
    double bp_mfrac = 1.0; // mask pixels per frame pixel a batch is sized for (the largest seen, + margin)
    int bp_bm_blocks = 0;
    int bp_F = 0, bp_err_frame = -1;
    int64_t bp_nnz = 0;
    std::vector<int32_t> bp_col, bp_label, bp_stats;
    std::vector<int64_t> bp_off;

    // ---- row-block sharding over processes ----
    int sh_rank = 0, sh_world = 1;
    int sh_pending = 0;          // MC_SHARD_* phase waiting for the host's exchange, 0 = none
    int sh_r0 = 0, sh_r1 = 0;    // this rank's S3 mask rows
    int64_t sh_s3_words = -1;    // size of this rank's S3 block (valid while sh_pending == MC_SHARD_S3)
    mc_graph_params sh_params{};
    DevBuf d_sh_eoff;
    // native collectives (mc_ctx_attach_comm / mc_ctx_comm_init): with a communicator attached the
    // sharded mc_graph_build / mc_cluster_run run their exchanges themselves, on the context stream
    void *comm = nullptr;        // ncclComm_t
    bool own_comm = false;
    DevBuf d_sh_send, d_sh_recv, d_sh_size;
    // S6 state kept across the FOREST exchange
    int s6_nthr = 0;
    bool s6_dense_obs = false;
    float s6_ctf = 0.f;
    // edge capture for the set-order replay (mc_cluster_set_edge_capture)
    int64_t cap_edges = 0;
    DevBuf d_cap_buf, d_cap_cnt;

    // ---- post-processing ----
    DevBuf d_pp_posmap;  // one P-entry position map per workgroup, -1 at rest
    int64_t pp_posmap_P = 0;
    int pp_posmap_slots = 0;
    bool have_pp = false;
    mc_pp_info pp_info{};
    std::vector<int32_t> pp_entry_obj, pp_qobj, pp_obj_node;
    std::vector<double> pp_qcov, pp_box;
    std::vector<uint8_t> pp_state;
};

namespace {

int fail(mc_ctx *ctx, const McError &e)
{
    if (ctx) ctx->err = e.msg;
    return e.code;
}

template <typename Fn>
int guarded(mc_ctx *ctx, Fn &&fn)
{
    if (!ctx) return MC_ERR_INVALID;
    try {
        MC_HIP(hipSetDevice(ctx->device));
        fn();
        return MC_OK;
    } catch (const McError &e) {
        return fail(ctx, e);
    } catch (const std::exception &e) {
        return fail(ctx, McError{MC_ERR_INVALID, e.what()});
    }
}

inline dim3 grid_for(int64_t n, int per_block = 256, int cap = 4096)
{
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return dim3(static_cast<unsigned>(g));
}

void sync_stats(mc_ctx *ctx)
{
    MC_HIP(hipMemcpyAsync(ctx->h_stats, ctx->d_stats.ptr, ST_COUNT * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    MC_HIP(hipStreamSynchronize(ctx->stream));
    ctx->timer.collect();
}


// S4 histogram launch: persistent blocks, R lane-indexed LDS replicas (odd stride)
// rng: >= ceil(M / 64) int2 of scratch
void launch_hist(hipStream_t s, const unsigned long long *vf, int M, int F, unsigned long long *hist, int2 *rng,
                 int shard_rank = 0, int shard_world = 1)
{
    if (!M || !F) return;
    const int FW = (F + 63) / 64;
    const int nblk = ceil_div(M, mc::kHistTile);
    hipLaunchKernelGGL(mc::k_s4_ranges, grid_for(static_cast<int64_t>(nblk) * 64), dim3(256), 0, s, vf, M, FW, nblk, rng);
    const long long ntiles = static_cast<long long>(nblk) * (nblk + 1) / 2;
    const int HS = (F + 1) | 1;
    int R = 32;
    while (R > 1 && static_cast<size_t>(R) * HS * 4 > 40 * 1024) R >>= 1;
    const size_t lds = 2 * mc::kHistTile * mc::kHistKW * sizeof(unsigned long long) + static_cast<size_t>(R) * HS * 4;
    const long long grid = std::min<long long>(ntiles, 1024);
    hipLaunchKernelGGL(mc::k_s4_hist, dim3(static_cast<unsigned>(grid)), dim3(256), lds, s, vf, M, FW, F, nblk, ntiles, R,
                       HS, rng, hist, shard_rank, shard_world);
}

// S3 work lists of this rank's mask rows [sh_r0, sh_r1) (all rows when not sharded): a wave per
// mask for the bulk, a workgroup per mask for large masks, largest first.  Rows are split over
// the ranks in contiguous blocks of about equal point counts.
void build_s3_lists(mc_ctx *ctx, const std::vector<int32_t> &frame_start)
{
    const int M = ctx->M, F = ctx->F;
    hipStream_t s = ctx->stream;
    {
        const int64_t tot = ctx->h_off[M];
        const int r = ctx->sh_rank, W = ctx->sh_world;
        auto cut = [&](int k) {  // first row whose cumulative points reach k/W of the total
            if (k <= 0) return 0;
            if (k >= W) return M;
            const int64_t target = (tot * k + W - 1) / W;
            return static_cast<int>(std::lower_bound(ctx->h_off.begin(), ctx->h_off.begin() + M + 1,
                                                     static_cast<int32_t>(target)) - ctx->h_off.begin());
        };
        ctx->sh_r0 = std::min(cut(r), M);
        ctx->sh_r1 = std::max(ctx->sh_r0, std::min(cut(r + 1), M));
    }
    int max_per_frame = 0;
    for (int c = 0; c < F; c++) max_per_frame = std::max(max_per_frame, frame_start[c + 1] - frame_start[c]);
    const bool wave_ok = F <= 64 * mc::kS3wFrameWords64 && max_per_frame < mc::kS3wCounters;
    std::vector<int> small, big;
    for (int g = ctx->sh_r0; g < ctx->sh_r1; g++) {
        const int sz = ctx->h_off[g + 1] - ctx->h_off[g];
        (wave_ok && sz <= mc::kS3SmallPts ? small : big).push_back(g);
    }
    // largest masks first: the long waves start early instead of forming the tail (a stable
    // counting sort by size, descending: std::stable_sort of C3's 81k rows took ~4 ms of host time)
    auto by_size_desc = [&](std::vector<int> &v) {
        if (v.size() < 2) return;
        int mx = 0;
        for (int g : v) mx = std::max(mx, ctx->h_off[g + 1] - ctx->h_off[g]);
        if (mx > (1 << 22)) {
            std::stable_sort(v.begin(), v.end(), [&](int x, int y) {
                return ctx->h_off[x + 1] - ctx->h_off[x] > ctx->h_off[y + 1] - ctx->h_off[y];
            });
            return;
        }
        std::vector<int> start(mx + 2, 0);
        for (int g : v) start[mx - (ctx->h_off[g + 1] - ctx->h_off[g]) + 1]++;
        for (int i = 1; i <= mx + 1; i++) start[i] += start[i - 1];
        std::vector<int> out(v.size());
        for (int g : v) out[start[mx - (ctx->h_off[g + 1] - ctx->h_off[g])]++] = g;
        v.swap(out);
    };
    by_size_desc(small);
    by_size_desc(big);
    ctx->n_s3_small = static_cast<int>(small.size());
    ctx->n_s3_big = static_cast<int>(big.size());
    ctx->d_s3_small.reserve((small.size() + 1) * sizeof(int));
    ctx->d_s3_big.reserve((big.size() + 1) * sizeof(int));
    if (!small.empty())
        MC_HIP(hipMemcpyAsync(ctx->d_s3_small.ptr, small.data(), small.size() * sizeof(int), hipMemcpyHostToDevice, s));
    if (!big.empty())
        MC_HIP(hipMemcpyAsync(ctx->d_s3_big.ptr, big.data(), big.size() * sizeof(int), hipMemcpyHostToDevice, s));
    MC_HIP(hipStreamSynchronize(s));
}

std::vector<int32_t> frame_starts(const mc_ctx *ctx)
{
    std::vector<int32_t> fs(ctx->F + 1, 0);
    int g = 0;
    for (int c = 0; c <= ctx->F; c++) {
        while (g < ctx->M && ctx->h_col[g] < c) g++;
        fs[c] = g;
    }
    return fs;
}

}  // namespace

static void shard_drain_native(mc_ctx *ctx);
static void comm_detach(mc_ctx *ctx);
namespace {
bool sharded(const mc_ctx *ctx);
}

extern "C" {

int mc_ctx_create(int device, mc_ctx **out)
{
    if (!out) return MC_ERR_INVALID;
    *out = nullptr;
    mc_ctx *ctx = new mc_ctx();
    ctx->device = device;
    int rc = guarded(ctx, [&] {
        MC_HIP(hipSetDevice(ctx->device));
        MC_HIP(hipDeviceGetAttribute(&ctx->num_cu, hipDeviceAttributeMultiprocessorCount, ctx->device));
        MC_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
        ctx->own_stream = true;
        MC_HIP(hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
        MC_HIP(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
        MC_HIP(hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
        for (int c = 0; c < mc::kBpStreamClasses; c++) {
            MC_HIP(hipStreamCreateWithFlags(&ctx->cls_stream[c], hipStreamNonBlocking));
            MC_HIP(hipEventCreateWithFlags(&ctx->ev_cls[c], hipEventDisableTiming));
        }
        MC_HIP(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_stats), ST_COUNT * sizeof(int), hipHostMallocDefault));
        ctx->d_stats.reserve(ST_COUNT * sizeof(int));
        MC_HIP(hipMemset(ctx->d_stats.ptr, 0, ST_COUNT * sizeof(int)));
    });
    if (rc != MC_OK) {
        mc_ctx_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return MC_OK;
}

void mc_ctx_destroy(mc_ctx *ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->comm) {
        try {
            comm_detach(ctx);
        } catch (const McError &) {
        }
    }
    DevBuf *bufs[] = {&ctx->d_mask_off, &ctx->d_mask_pts, &ctx->d_mask_col, &ctx->d_mask_label, &ctx->d_frame_start,
                      &ctx->d_valid, &ctx->d_deg, &ctx->d_pt_off, &ctx->d_pt_list, &ctx->d_boundary,
                      &ctx->d_pfm, &ctx->d_scan_tmp, &ctx->d_ctmp, &ctx->d_crow_len, &ctx->d_useg, &ctx->d_keep_cnt,
                      &ctx->d_node_flag, &ctx->d_node_pos, &ctx->d_c_off, &ctx->d_c_idx, &ctx->d_vf, &ctx->d_hist, &ctx->d_s4rng,
                      &ctx->d_thr, &ctx->d_isint, &ctx->d_stats, &ctx->d_node0_g, &ctx->d_n0_off, &ctx->d_n0_len,
                      &ctx->d_n0_ptoff, &ctx->d_n0_ptlen, &ctx->d_n0_vf, &ctx->d_user_cidx, &ctx->d_user_pts,
                      &ctx->d_parent, &ctx->d_root, &ctx->d_isroot, &ctx->d_rank, &ctx->d_label, &ctx->d_levels,
                      &ctx->d_memcnt, &ctx->d_memoff, &ctx->d_ublen, &ctx->d_newoff, &ctx->d_members, &ctx->d_colcnt,
                      &ctx->d_coloff, &ctx->d_colnodes, &ctx->d_ovf_n, &ctx->d_scratch,
                      &ctx->d_touched, &ctx->d_edges, &ctx->d_spread, &ctx->d_Nlev, &ctx->d_final_label,
                      &ctx->d_poolA, &ctx->d_poolB, &ctx->d_offA, &ctx->d_offB, &ctx->d_lenA, &ctx->d_lenB,
                      &ctx->d_vfA, &ctx->d_vfB, &ctx->d_pmin, &ctx->d_pmax, &ctx->d_nwords, &ctx->d_woff,
                      &ctx->d_bm, &ctx->d_ptcnt, &ctx->d_ptoff_out, &ctx->d_pts_out, &ctx->d_owner0,
                      &ctx->d_node_of_mask, &ctx->d_ownA, &ctx->d_ownB, &ctx->d_cap, &ctx->d_obj_of_mask,
                      &ctx->d_s3_small, &ctx->d_s3_big, &ctx->d_collen, &ctx->d_sh_eoff, &ctx->d_sh_send, &ctx->d_sh_recv, &ctx->d_sh_size,
                      &ctx->d_cap_buf, &ctx->d_cap_cnt};
    for (DevBuf *b : bufs) b->release();
    DevBuf *bp_bufs[] = {&ctx->d_scene, &ctx->d_gcnt, &ctx->d_gstart, &ctx->d_gbkt, &ctx->d_gcellk, &ctx->d_gpts,
                         &ctx->d_gidx, &ctx->d_gcell, &ctx->d_gscan_tmp, &ctx->d_in_depth, &ctx->d_in_seg, &ctx->d_in_raw,
                         &ctx->d_in_intr, &ctx->d_in_pose, &ctx->d_band, &ctx->d_bpvid, &ctx->d_present, &ctx->d_fflags,
                         &ctx->d_cand, &ctx->d_npix, &ctx->d_csidx, &ctx->d_poff, &ctx->d_slot_of, &ctx->d_bpstat,
                         &ctx->d_slot_frame, &ctx->d_slot_id, &ctx->d_slot_np, &ctx->d_slot_pix, &ctx->d_slot_nv,
                         &ctx->d_slot_m, &ctx->d_slot_ns, &ctx->d_slot_box, &ctx->d_slot_nn, &ctx->d_slot_toff,
                         &ctx->d_slot_cov, &ctx->d_pix_list, &ctx->d_hkey, &ctx->d_hfirst,
                         &ctx->d_vox_entry, &ctx->d_vpts, &ctx->d_pcell, &ctx->d_pbkt, &ctx->d_bcnt,
                         &ctx->d_bstart, &ctx->d_blist, &ctx->d_ncnt, &ctx->d_par, &ctx->d_droot, &ctx->d_rnk,
                         &ctx->d_lab, &ctx->d_ccnt, &ctx->d_ssidx, &ctx->d_avg, &ctx->d_qpts, &ctx->d_bpbm, &ctx->d_tmp,
                         &ctx->d_kflag, &ctx->d_ksize, &ctx->d_midx, &ctx->d_moff, &ctx->d_out_col,
                         &ctx->d_out_label, &ctx->d_out_off, &ctx->d_out_pts, &ctx->d_bp_pts,
                         &ctx->d_cls_list, &ctx->d_nbl, &ctx->d_lean, &ctx->d_vox_order,
                         &ctx->d_vx_pvid, &ctx->d_vx_list, &ctx->d_vx_fb, &ctx->d_bppack, &ctx->d_acc, &ctx->d_hvid,
                         &ctx->d_slot_grid, &ctx->d_scanm};
    for (DevBuf *b : bp_bufs) b->release();
    if (ctx->copy) (void)hipStreamSynchronize(ctx->copy), (void)hipStreamDestroy(ctx->copy);
    if (ctx->ev_up) (void)hipEventDestroy(ctx->ev_up);
    if (ctx->h_stats) (void)hipHostFree(ctx->h_stats);
    if (ctx->h_bppack) (void)hipHostFree(ctx->h_bppack);
    if (ctx->h_bpstat) (void)hipHostFree(ctx->h_bpstat);
    if (ctx->ev_pack) (void)hipEventDestroy(ctx->ev_pack);
    for (int b = 0; b < 2; b++) {
        if (ctx->h_stage[b]) (void)hipHostFree(ctx->h_stage[b]);
        if (ctx->ev_stage[b]) (void)hipEventDestroy(ctx->ev_stage[b]);
    }
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->side) (void)hipStreamSynchronize(ctx->side), (void)hipStreamDestroy(ctx->side);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    for (int c = 0; c < mc::kBpStreamClasses; c++) {
        if (ctx->cls_stream[c]) (void)hipStreamSynchronize(ctx->cls_stream[c]), (void)hipStreamDestroy(ctx->cls_stream[c]);
        if (ctx->ev_cls[c]) (void)hipEventDestroy(ctx->ev_cls[c]);
    }
    delete ctx;
}

int mc_ctx_set_stream(mc_ctx *ctx, void *hip_stream)
{
    return guarded(ctx, [&] {
        MC_HIP(hipStreamSynchronize(ctx->stream));
        if (ctx->own_stream) MC_HIP(hipStreamDestroy(ctx->stream));
        if (hip_stream) {
            ctx->stream = static_cast<hipStream_t>(hip_stream);
            ctx->own_stream = false;
        } else {
            MC_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
            ctx->own_stream = true;
        }
    });
}

void *mc_ctx_get_stream(mc_ctx *ctx) { return ctx ? static_cast<void *>(ctx->stream) : nullptr; }

int mc_ctx_synchronize(mc_ctx *ctx)
{
    return guarded(ctx, [&] {
        MC_HIP(hipStreamSynchronize(ctx->stream));
        ctx->timer.collect();
    });
}

const char *mc_ctx_last_error(mc_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int mc_ctx_set_timing(mc_ctx *ctx, int enable)
{
    return guarded(ctx, [&] {
        MC_HIP(hipStreamSynchronize(ctx->stream));
        ctx->timer.collect();
        ctx->timer.enabled = enable != 0;
    });
}

int mc_ctx_set_timing_filter(mc_ctx *ctx, const char *kernel)
{
    return guarded(ctx, [&] {
        MC_HIP(hipStreamSynchronize(ctx->stream));
        ctx->timer.collect();
        ctx->timer.filter = kernel ? kernel : "";
    });
}

int mc_ctx_get_kernel_time(mc_ctx *ctx, const char *kernel, double *total_ms, int64_t *launches)
{
    return guarded(ctx, [&] {
        MC_HIP(hipStreamSynchronize(ctx->stream));
        ctx->timer.collect();
        auto it = ctx->timer.totals.find(kernel ? kernel : "");
        if (total_ms) *total_ms = it == ctx->timer.totals.end() ? 0.0 : it->second.first;
        if (launches) *launches = it == ctx->timer.totals.end() ? 0 : it->second.second;
    });
}

int mc_ctx_reset_kernel_times(mc_ctx *ctx)
{
    return guarded(ctx, [&] {
        MC_HIP(hipStreamSynchronize(ctx->stream));
        ctx->timer.collect();
        ctx->timer.totals.clear();
    });
}

int mc_ctx_set_memory_budget(mc_ctx *ctx, int64_t bytes)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(bytes >= 0, MC_ERR_INVALID, "negative memory budget");
        ctx->mem_budget = bytes;
    });
}

int mc_debug_counters(mc_ctx *ctx, int64_t *out, int32_t n, int reset)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(out && n >= 1 && n <= 9, MC_ERR_INVALID, "bad counter array");
        MC_HIP(hipDeviceSynchronize());
        unsigned long long c[8] = {};
        MC_HIP(hipMemcpyFromSymbol(c, HIP_SYMBOL(mc::g_bp_dbg), sizeof(c)));
        out[0] = MC_DBG_CHECK ? 1 : 0;
        for (int k = 1; k < n; k++) out[k] = static_cast<int64_t>(c[k - 1]);
        if (reset) {
            const unsigned long long z[8] = {};
            const unsigned zp = 0;
            MC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(mc::g_bp_dbg), z, sizeof(z)));
            MC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(mc::g_bp_dbg_printed), &zp, sizeof(zp)));
        }
    });
}

// ---------------------------------------------------------------------------------------------
// scene input
// ---------------------------------------------------------------------------------------------
__global__ void k_validate_pts(const int *pts, int nnz, int64_t P, int *bad)
{
    for (int i = blockIdx.x * 256 + threadIdx.x; i < nnz; i += gridDim.x * 256)
        if (pts[i] < 0 || pts[i] >= P) atomicOr(bad, 1);
}

int mc_scene_set_masks(mc_ctx *ctx, int64_t num_points, int32_t num_frames, int32_t num_masks_in,
                       const int32_t *mask_col, const int32_t *mask_label, const int64_t *mask_off,
                       const int32_t *mask_pts, int pts_on_device)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(num_points >= 0 && num_points < (int64_t(1) << 31) - 1, MC_ERR_UNSUPPORTED, "num_points out of range");
        MC_REQUIRE(num_frames >= 0 && num_frames <= 16384, MC_ERR_UNSUPPORTED, "num_frames must be <= 16384");
        MC_REQUIRE(num_masks_in >= 0, MC_ERR_INVALID, "num_masks < 0");
        MC_REQUIRE(num_masks_in == 0 || (mask_col && mask_label && mask_off), MC_ERR_INVALID, "null mask arrays");
        MC_REQUIRE(!mask_off || mask_off[0] == 0, MC_ERR_INVALID, "mask_off[0] != 0");
        const int64_t nnz = num_masks_in ? mask_off[num_masks_in] : 0;
        MC_REQUIRE(nnz < (int64_t(1) << 31) - 1, MC_ERR_UNSUPPORTED, "more than 2^31 mask points");
        MC_REQUIRE(nnz == 0 || mask_pts, MC_ERR_INVALID, "null mask_pts");
        ctx->have_scene = ctx->have_graph = ctx->have_nodes = ctx->have_cluster = false;
        ctx->P = num_points;
        ctx->F = num_frames;
        ctx->FW = (num_frames + 63) / 64;
        ctx->M_in = num_masks_in;
        // validation + the frame-skip rule (construction.py:50-51)
        std::vector<int64_t> frame_pts(std::max(1, num_frames), 0);
        std::vector<int> frame_masks(std::max(1, num_frames), 0);
        for (int g = 0; g < num_masks_in; g++) {
            const int c = mask_col[g];
            MC_REQUIRE(c >= 0 && c < num_frames, MC_ERR_INVALID, "mask_col out of range");
            MC_REQUIRE(g == 0 || mask_col[g - 1] <= c, MC_ERR_INVALID, "mask_col must be non-decreasing");
            MC_REQUIRE(mask_label[g] >= 1 && mask_label[g] <= 65535, MC_ERR_INVALID, "mask label must be in [1, 65535]");
            MC_REQUIRE(mask_off[g + 1] >= mask_off[g], MC_ERR_INVALID, "mask_off must be non-decreasing");
            frame_pts[c] += mask_off[g + 1] - mask_off[g];
            frame_masks[c]++;
            MC_REQUIRE(frame_masks[c] < 2048, MC_ERR_UNSUPPORTED, "more than 2047 masks in a frame");
        }
        {
            std::vector<int> seen(65536, -1);
            for (int g = 0; g < num_masks_in; g++) {
                MC_REQUIRE(seen[mask_label[g]] != mask_col[g], MC_ERR_INVALID, "duplicate mask label within a frame");
                seen[mask_label[g]] = mask_col[g];
            }
        }
        ctx->h_col.clear();
        ctx->h_label.clear();
        ctx->h_in_index.clear();
        ctx->h_off.assign(1, 0);
        for (int g = 0; g < num_masks_in; g++) {
            if (frame_pts[mask_col[g]] == 0) continue;  // masks of a skipped frame have no points
            ctx->h_in_index.push_back(g);
            ctx->h_col.push_back(mask_col[g]);
            ctx->h_label.push_back(mask_label[g]);
            ctx->h_off.push_back(static_cast<int32_t>(mask_off[g + 1]));
        }
        const int M = static_cast<int>(ctx->h_col.size());
        ctx->M = M;
        ctx->nnz = static_cast<int>(nnz);
        MC_REQUIRE(M <= 262144, MC_ERR_UNSUPPORTED, "more than 262144 global masks");
        std::vector<int32_t> frame_start(num_frames + 1, 0);
        {
            int g = 0;
            for (int c = 0; c <= num_frames; c++) {
                while (g < M && ctx->h_col[g] < c) g++;
                frame_start[c] = g;
            }
        }
        const int64_t P = num_points;
        const int F = num_frames, FW = ctx->FW;
        hipStream_t s = ctx->stream;
        ctx->d_mask_off.reserve((M + 1) * sizeof(int));
        ctx->d_mask_col.reserve((M + 1) * sizeof(int));
        ctx->d_mask_label.reserve((M + 1) * sizeof(int));
        ctx->d_frame_start.reserve((F + 2) * sizeof(int));
        ctx->d_mask_pts.reserve((nnz + 1) * sizeof(int));
        ctx->d_valid.reserve(sizeof(int));
        MC_HIP(hipMemcpyAsync(ctx->d_mask_off.ptr, ctx->h_off.data(), (M + 1) * sizeof(int), hipMemcpyHostToDevice, s));
        if (M) {
            MC_HIP(hipMemcpyAsync(ctx->d_mask_col.ptr, ctx->h_col.data(), M * sizeof(int), hipMemcpyHostToDevice, s));
            MC_HIP(hipMemcpyAsync(ctx->d_mask_label.ptr, ctx->h_label.data(), M * sizeof(int), hipMemcpyHostToDevice, s));
        }
        MC_HIP(hipMemcpyAsync(ctx->d_frame_start.ptr, frame_start.data(), (F + 1) * sizeof(int), hipMemcpyHostToDevice, s));
        if (nnz)
            MC_HIP(hipMemcpyAsync(ctx->d_mask_pts.ptr, mask_pts, nnz * sizeof(int),
                                  pts_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
        MC_HIP(hipMemsetAsync(ctx->d_valid.ptr, 0, sizeof(int), s));
        if (nnz)
            hipLaunchKernelGGL(k_validate_pts, grid_for(nnz), dim3(256), 0, s, ctx->d_mask_pts.as<int>(),
                               static_cast<int>(nnz), P, ctx->d_valid.as<int>());
        int bad = 0;
        MC_HIP(hipMemcpyAsync(&bad, ctx->d_valid.ptr, sizeof(int), hipMemcpyDeviceToHost, s));
        MC_HIP(hipStreamSynchronize(s));
        MC_REQUIRE(bad == 0, MC_ERR_INVALID, "mask point id out of [0, num_points)");

        // S2/S3/S4 buffers (allocated once per scene; nothing is allocated while building)
        ctx->d_deg.reserve((P + 1) * sizeof(int));
        ctx->d_spread.reserve(mc::kSpread * mc::kSpreadStrideI * sizeof(int));
        MC_HIP(hipMemsetAsync(ctx->d_deg.ptr, 0, (P + 1) * sizeof(int), s));  // kept zero by the S2 scatter
        ctx->d_pt_off.reserve((P + 2) * sizeof(int));
        ctx->d_pt_list.reserve((nnz + 1) * sizeof(unsigned));
        ctx->d_boundary.reserve(P + 1);
        ctx->d_pfm.reserve((P * FW + 1) * sizeof(unsigned long long));
        ctx->d_scan_tmp.reserve((2 * (P / 4096 + 4) + 16) * sizeof(int));
        ctx->d_ctmp.reserve((static_cast<size_t>(M) * F + 1) * sizeof(int));
        ctx->d_crow_len.reserve((M + 1) * sizeof(int));
        ctx->d_useg.reserve(M + 1);
        ctx->d_keep_cnt.reserve((M + 1) * sizeof(int));
        ctx->d_node_flag.reserve((M + 1) * sizeof(int));
        ctx->d_node_pos.reserve((M + 2) * sizeof(int));
        ctx->d_c_off.reserve((M + 2) * sizeof(int));
        ctx->d_c_idx.reserve((static_cast<size_t>(M) * F + 1) * sizeof(int));
        ctx->d_vf.reserve((static_cast<size_t>(M) * FW + 1) * sizeof(unsigned long long));
        ctx->d_hist.reserve((F + 2) * sizeof(unsigned long long));
        ctx->d_s4rng.reserve((M / 64 + 2) * sizeof(int2));
        ctx->d_thr.reserve(32 * sizeof(float));
        ctx->d_isint.reserve(32 * sizeof(int));
        ctx->d_node0_g.reserve((M + 1) * sizeof(int));
        ctx->d_n0_off.reserve((M + 1) * sizeof(int));
        ctx->d_n0_len.reserve((M + 1) * sizeof(int));
        ctx->d_n0_ptoff.reserve((M + 1) * sizeof(int));
        ctx->d_n0_ptlen.reserve((M + 1) * sizeof(int));
        ctx->d_n0_vf.reserve((static_cast<size_t>(M) * FW + 1) * sizeof(unsigned long long));
        ctx->d_owner0.reserve((static_cast<size_t>(M) * F + 1) * sizeof(int));
        ctx->d_node_of_mask.reserve((M + 1) * sizeof(int));
        ctx->d_obj_of_mask.reserve((M + 1) * sizeof(int));
        build_s3_lists(ctx, frame_start);
        ctx->have_scene = true;
    });
}

// ---------------------------------------------------------------------------------------------
// S2–S5
// ---------------------------------------------------------------------------------------------
// S3 undo + S5 + S4 (this rank's tiles of the observer histogram when sharded)
static void graph_build_tail(mc_ctx *ctx)
{
    hipStream_t s = ctx->stream;
    const int F = ctx->F, FW = ctx->FW, M = ctx->M;
    int *stats = ctx->d_stats.as<int>();
    if (M) {  // S3 undo + S5
        TimedScope ts(ctx->timer, s, "s3_undo_s5");
        hipLaunchKernelGGL(mc::k_s3_undo_count, dim3(ceil_div(std::max(M, F + 1), 256)), dim3(256), 0, s,
                           ctx->d_ctmp.as<int>(), ctx->d_crow_len.as<int>(), ctx->d_useg.as<unsigned char>(), M, F,
                           ctx->d_keep_cnt.as<int>(), ctx->d_node_flag.as<int>(),
                           ctx->d_hist.as<unsigned long long>(), ctx->d_spread.as<int>(), stats + ST_NBND);
        mc::scan_device_n(s, ctx->d_keep_cnt.as<int>(), ctx->d_c_off.as<int>(), nullptr, M, stats + ST_NNZC,
                          ctx->d_node_flag.as<int>(), ctx->d_node_pos.as<int>(), stats + ST_N0);
        hipLaunchKernelGGL(mc::k_s3_undo_write, dim3(ceil_div(M, 256)), dim3(256), 0, s, ctx->d_ctmp.as<int>(),
                           ctx->d_crow_len.as<int>(), ctx->d_useg.as<unsigned char>(), ctx->d_mask_col.as<int>(), M,
                           F, FW, ctx->d_c_off.as<int>(), ctx->d_c_idx.as<int>(),
                           ctx->d_vf.as<unsigned long long>());
        hipLaunchKernelGGL(mc::k_s5_nodes, dim3(ceil_div(M, 256)), dim3(256), 0, s, ctx->d_node_pos.as<int>(),
                           ctx->d_useg.as<unsigned char>(), ctx->d_c_off.as<int>(), ctx->d_mask_off.as<int>(),
                           ctx->d_vf.as<unsigned long long>(), M, FW, ctx->d_node0_g.as<int>(),
                           ctx->d_n0_off.as<int>(), ctx->d_n0_len.as<int>(), ctx->d_n0_ptoff.as<int>(),
                           ctx->d_n0_ptlen.as<int>(), ctx->d_n0_vf.as<unsigned long long>(),
                           ctx->d_owner0.as<int>(), ctx->d_node_of_mask.as<int>());
    } else {
        MC_HIP(hipMemsetAsync(ctx->d_hist.ptr, 0, (F + 1) * sizeof(unsigned long long), s));
    }
    {  // S4: observer histogram (the thresholds follow in graph_build_thresholds)
        TimedScope ts(ctx->timer, s, "s4_observer_hist");
        launch_hist(s, ctx->d_vf.as<unsigned long long>(), M, F, ctx->d_hist.as<unsigned long long>(),
                    ctx->d_s4rng.as<int2>(), ctx->sh_rank, ctx->sh_world);
    }
    MC_HIP(hipGetLastError());
}

static void graph_build_thresholds(mc_ctx *ctx)
{
    hipStream_t s = ctx->stream;
    const int F = ctx->F;
    int *stats = ctx->d_stats.as<int>();
    {
        TimedScope ts(ctx->timer, s, "s4_observer_hist");
        hipLaunchKernelGGL(mc::k_s4_thresholds, dim3(1), dim3(256), (F + 1) * sizeof(unsigned long long), s,
                           ctx->d_hist.as<unsigned long long>(), F, ctx->d_thr.as<float>(), ctx->d_isint.as<int>(),
                           stats + ST_NTHR, stats + ST_THR_STATUS);
    }
    MC_HIP(hipGetLastError());
    // level-0 nodes live in the graph's buffers
    ctx->n0_pool = ctx->d_c_idx.as<int>();
    ctx->n0_pts = ctx->d_mask_pts.as<int>();
    ctx->Mn = ctx->M;
    ctx->n0_pts_total = ctx->nnz;
    ctx->nodes_from_graph = true;
    ctx->have_graph = true;
    ctx->have_nodes = true;
}

int mc_graph_build(mc_ctx *ctx, const mc_graph_params *params)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_scene, MC_ERR_STATE, "mc_graph_build before mc_scene_set_masks");
        MC_REQUIRE(params, MC_ERR_INVALID, "null params");
        hipStream_t s = ctx->stream;
        const int64_t P = ctx->P;
        const int F = ctx->F, FW = ctx->FW, M = ctx->M, nnz = ctx->nnz;
        int *stats = ctx->d_stats.as<int>();
        ctx->have_cluster = false;
        ctx->have_graph = ctx->have_nodes = false;
        ctx->sh_pending = 0;
        ctx->sh_params = *params;
        {  // S2
            TimedScope ts(ctx->timer, s, "s2_point_lists");
            hipLaunchKernelGGL(mc::k_s2_degree, grid_for(nnz), dim3(256), 0, s, ctx->d_mask_pts.as<int>(), nnz,
                               ctx->d_deg.as<int>(), stats, static_cast<int>(ST_COUNT), ctx->d_spread.as<int>());
            mc::scan_large(s, ctx->d_deg.as<int>(), ctx->d_pt_off.as<int>(), static_cast<int>(P), ctx->d_scan_tmp.as<int>());
            if (M)
                hipLaunchKernelGGL(mc::k_s2_scatter, dim3(M), dim3(256), 0, s, ctx->d_mask_off.as<int>(),
                                   ctx->d_mask_pts.as<int>(), ctx->d_mask_col.as<int>(), ctx->d_frame_start.as<int>(),
                                   ctx->d_pt_off.as<int>(), ctx->d_deg.as<int>(), ctx->d_pt_list.as<unsigned>());
            if (P)
                hipLaunchKernelGGL(mc::k_s2_points, dim3(ceil_div(P, 256)), dim3(256), 0, s, ctx->d_pt_off.as<int>(),
                                   ctx->d_pt_list.as<unsigned>(), static_cast<int>(P), FW,
                                   ctx->d_boundary.as<unsigned char>(), ctx->d_pfm.as<unsigned long long>(),
                                   ctx->d_spread.as<int>());
        }
        if (M) {  // S3
            TimedScope ts(ctx->timer, s, "s3_masks");
            // large masks (workgroup per mask) on the side stream, concurrent with the wave kernel
            const bool fork = ctx->n_s3_big && ctx->n_s3_small;
            if (fork) {
                MC_HIP(hipEventRecord(ctx->ev_fork, s));
                MC_HIP(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
            }
            if (ctx->n_s3_big)
                hipLaunchKernelGGL(mc::k_s3_masks<mc::kS3BigW>, grid_for(ctx->n_s3_big, 1, 8192),
                                   dim3(mc::S3Cfg<mc::kS3BigW>::NT), 0,
                                   fork ? ctx->side : s,
                                   ctx->d_s3_big.as<int>(), ctx->n_s3_big, ctx->d_mask_off.as<int>(),
                                   ctx->d_mask_pts.as<int>(), ctx->d_pt_off.as<int>(), ctx->d_pt_list.as<unsigned>(),
                                   ctx->d_boundary.as<unsigned char>(), ctx->d_pfm.as<unsigned long long>(), FW,
                                   ctx->d_frame_start.as<int>(), ctx->d_mask_label.as<int>(), F,
                                   params->mask_visible_threshold, params->contained_threshold,
                                   params->undersegment_filter_threshold, ctx->d_ctmp.as<int>(),
                                   ctx->d_crow_len.as<int>(), ctx->d_useg.as<unsigned char>());
            if (ctx->n_s3_small)
                hipLaunchKernelGGL(mc::k_s3_masks<1>, grid_for(ctx->n_s3_small, 4, 16384), dim3(256), 0, s,
                                   ctx->d_s3_small.as<int>(), ctx->n_s3_small, ctx->d_mask_off.as<int>(),
                                   ctx->d_mask_pts.as<int>(), ctx->d_pt_off.as<int>(), ctx->d_pt_list.as<unsigned>(),
                                   ctx->d_boundary.as<unsigned char>(), ctx->d_pfm.as<unsigned long long>(), FW,
                                   ctx->d_frame_start.as<int>(), ctx->d_mask_label.as<int>(), F,
                                   params->mask_visible_threshold, params->contained_threshold,
                                   params->undersegment_filter_threshold, ctx->d_ctmp.as<int>(),
                                   ctx->d_crow_len.as<int>(), ctx->d_useg.as<unsigned char>());
            if (fork) {
                MC_HIP(hipEventRecord(ctx->ev_join, ctx->side));
                MC_HIP(hipStreamWaitEvent(s, ctx->ev_join, 0));
            }
        }
        if (sharded(ctx)) {  // this rank's S3 rows go to the others first (mc_shard_export/import)
            ctx->sh_pending = MC_SHARD_S3;
            ctx->sh_s3_words = -1;
            if (ctx->comm) shard_drain_native(ctx);  // S3 rows, then the histogram, over RCCL
            return;
        }
        graph_build_tail(ctx);
        graph_build_thresholds(ctx);
    });
}

int mc_graph_get_info(mc_ctx *ctx, mc_graph_info *info)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_graph && info, MC_ERR_STATE, "no graph");
        sync_stats(ctx);
        const int *h = ctx->h_stats;
        info->num_points = ctx->P;
        info->num_frames = ctx->F;
        info->num_masks = ctx->M;
        info->num_nodes0 = h[ST_N0];
        info->num_undersegment = ctx->M - h[ST_N0];
        info->num_contained = h[ST_NNZC];
        info->num_boundary = h[ST_NBND];
        info->num_thresholds = h[ST_NTHR];
        info->threshold_status = h[ST_THR_STATUS];
    });
}

int mc_graph_get_global_masks(mc_ctx *ctx, int32_t *input_index)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_scene, MC_ERR_STATE, "no scene");
        std::copy(ctx->h_in_index.begin(), ctx->h_in_index.end(), input_index);
    });
}

int mc_graph_get_boundary(mc_ctx *ctx, uint8_t *flags)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_graph, MC_ERR_STATE, "no graph");
        if (ctx->P) MC_HIP(hipMemcpyAsync(flags, ctx->d_boundary.ptr, ctx->P, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int mc_graph_get_point_in_mask(mc_ctx *ctx, uint16_t *pim)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_graph, MC_ERR_STATE, "no graph");
        const size_t bytes = static_cast<size_t>(ctx->P) * ctx->F * sizeof(uint16_t);
        if (!bytes) return;
        DevBuf tmp;
        tmp.reserve(bytes);
        MC_HIP(hipMemsetAsync(tmp.ptr, 0, bytes, ctx->stream));
        hipLaunchKernelGGL(mc::k_s2_dense_pim, dim3(ceil_div(ctx->P, 256)), dim3(256), 0, ctx->stream,
                           ctx->d_pt_off.as<int>(), ctx->d_pt_list.as<unsigned>(), ctx->d_mask_label.as<int>(),
                           ctx->d_frame_start.as<int>(), static_cast<int>(ctx->P), ctx->F, tmp.as<unsigned short>());
        MC_HIP(hipMemcpyAsync(pim, tmp.ptr, bytes, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
        tmp.release();
    });
}

int mc_graph_get_point_frame_bits(mc_ctx *ctx, uint64_t *bits)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_graph, MC_ERR_STATE, "no graph");
        const size_t bytes = static_cast<size_t>(ctx->P) * ctx->FW * 8;
        if (bytes) MC_HIP(hipMemcpyAsync(bits, ctx->d_pfm.ptr, bytes, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int mc_graph_get_visible_frame_bits(mc_ctx *ctx, uint64_t *bits)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_graph, MC_ERR_STATE, "no graph");
        const size_t bytes = static_cast<size_t>(ctx->M) * ctx->FW * 8;
        if (bytes) MC_HIP(hipMemcpyAsync(bits, ctx->d_vf.ptr, bytes, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int mc_graph_get_contained(mc_ctx *ctx, int64_t *row_off, int32_t *col_idx)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_graph, MC_ERR_STATE, "no graph");
        sync_stats(ctx);
        std::vector<int32_t> off(ctx->M + 1);
        MC_HIP(hipMemcpyAsync(off.data(), ctx->d_c_off.ptr, (ctx->M + 1) * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        const int nnzc = ctx->h_stats[ST_NNZC];
        if (nnzc) MC_HIP(hipMemcpyAsync(col_idx, ctx->d_c_idx.ptr, nnzc * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
        for (int i = 0; i <= ctx->M; i++) row_off[i] = ctx->M ? off[i] : 0;
    });
}

int mc_graph_get_undersegment(mc_ctx *ctx, int32_t *ids)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_graph, MC_ERR_STATE, "no graph");
        std::vector<uint8_t> u(ctx->M);
        if (ctx->M) MC_HIP(hipMemcpyAsync(u.data(), ctx->d_useg.ptr, ctx->M, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
        int k = 0;
        for (int g = 0; g < ctx->M; g++)
            if (u[g]) ids[k++] = g;
    });
}

int mc_graph_get_nodes0(mc_ctx *ctx, int32_t *mask_index)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_graph, MC_ERR_STATE, "no graph");
        sync_stats(ctx);
        const int n0 = ctx->h_stats[ST_N0];
        if (n0) MC_HIP(hipMemcpyAsync(mask_index, ctx->d_node0_g.ptr, n0 * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int mc_graph_get_observer_hist(mc_ctx *ctx, uint64_t *hist)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_graph, MC_ERR_STATE, "no graph");
        MC_HIP(hipMemcpyAsync(hist, ctx->d_hist.ptr, (ctx->F + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int mc_graph_get_thresholds(mc_ctx *ctx, float *thr, int32_t *is_int, int32_t *n)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_graph, MC_ERR_STATE, "no graph");
        sync_stats(ctx);
        MC_HIP(hipMemcpyAsync(thr, ctx->d_thr.ptr, mc::kMaxThresholds * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipMemcpyAsync(is_int, ctx->d_isint.ptr, mc::kMaxThresholds * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
        *n = ctx->h_stats[ST_NTHR];
        if (ctx->h_stats[ST_THR_STATUS] != MC_OK)
            throw McError{ctx->h_stats[ST_THR_STATUS], "no positive observer count (np.percentile of an empty array)"};
    });
}

int mc_observer_thresholds(mc_ctx *ctx, int32_t num_rows, int32_t num_frames, const uint64_t *vf_bits, float *thr,
                           int32_t *is_int, int32_t *n)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(num_rows >= 0 && num_frames >= 0 && num_frames <= 16384, MC_ERR_INVALID, "bad sizes");
        MC_REQUIRE(thr && is_int && n && (num_rows == 0 || num_frames == 0 || vf_bits), MC_ERR_INVALID, "null argument");
        hipStream_t s = ctx->stream;
        const int M = num_rows, F = num_frames, FW = (F + 63) / 64;
        DevBuf vf, hist, dthr, disint, st;
        vf.reserve(static_cast<size_t>(M) * FW * 8 + 8);
        hist.reserve((F + 2) * 8);
        dthr.reserve(32 * 4);
        disint.reserve(32 * 4);
        st.reserve(2 * 4);
        if (M && FW) MC_HIP(hipMemcpyAsync(vf.ptr, vf_bits, static_cast<size_t>(M) * FW * 8, hipMemcpyHostToDevice, s));
        MC_HIP(hipMemsetAsync(hist.ptr, 0, (F + 1) * 8, s));
        DevBuf rng;
        rng.reserve((M / 64 + 2) * sizeof(int2));
        launch_hist(s, vf.as<unsigned long long>(), M, F, hist.as<unsigned long long>(), rng.as<int2>());
        hipLaunchKernelGGL(mc::k_s4_thresholds, dim3(1), dim3(256), (F + 1) * sizeof(unsigned long long), s,
                           hist.as<unsigned long long>(), F,
                           dthr.as<float>(), disint.as<int>(), st.as<int>(), st.as<int>() + 1);
        int hs[2];
        MC_HIP(hipMemcpyAsync(hs, st.ptr, 8, hipMemcpyDeviceToHost, s));
        MC_HIP(hipMemcpyAsync(thr, dthr.ptr, mc::kMaxThresholds * 4, hipMemcpyDeviceToHost, s));
        MC_HIP(hipMemcpyAsync(is_int, disint.ptr, mc::kMaxThresholds * 4, hipMemcpyDeviceToHost, s));
        MC_HIP(hipStreamSynchronize(s));
        *n = hs[0];
        if (hs[1] != MC_OK) throw McError{hs[1], "no positive observer count (np.percentile of an empty array)"};
    });
}

// ---------------------------------------------------------------------------------------------
// arbitrary level-0 nodes
// ---------------------------------------------------------------------------------------------
__global__ void k_nodes_from_csr(int n, const int64_t *c_off, const int64_t *pt_off, int *n_off, int *n_len, int *n_ptoff,
                                 int *n_ptlen, int *owner)
{
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        n_off[i] = static_cast<int>(c_off[i]);
        n_len[i] = static_cast<int>(c_off[i + 1] - c_off[i]);
        n_ptoff[i] = static_cast<int>(pt_off[i]);
        n_ptlen[i] = static_cast<int>(pt_off[i + 1] - pt_off[i]);
        for (int64_t e = c_off[i]; e < c_off[i + 1]; e++) owner[e] = i;
    }
}

int mc_nodes_set(mc_ctx *ctx, int32_t num_nodes, int32_t num_frames, int32_t num_masks, int64_t num_points,
                 const uint64_t *vf_bits, const int64_t *c_off, const int32_t *c_idx, const int64_t *pt_off,
                 const int32_t *pt_idx)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(num_nodes >= 0 && num_frames >= 0 && num_masks >= 0 && num_points >= 0, MC_ERR_INVALID, "negative size");
        MC_REQUIRE(num_frames <= 16384, MC_ERR_UNSUPPORTED, "num_frames must be <= 16384");
        MC_REQUIRE(num_masks <= 262144, MC_ERR_UNSUPPORTED, "num_masks must be <= 262144");
        MC_REQUIRE(num_nodes == 0 || (vf_bits && c_off && pt_off), MC_ERR_INVALID, "null node arrays");
        const int64_t nc = num_nodes ? c_off[num_nodes] : 0, np = num_nodes ? pt_off[num_nodes] : 0;
        MC_REQUIRE(nc < (int64_t(1) << 31) && np < (int64_t(1) << 31), MC_ERR_UNSUPPORTED, "node arrays too large");
        for (int64_t i = 0; i < nc; i++) MC_REQUIRE(c_idx[i] >= 0 && c_idx[i] < num_masks, MC_ERR_INVALID, "contained id out of range");
        for (int64_t i = 0; i < np; i++) MC_REQUIRE(pt_idx[i] >= 0 && pt_idx[i] < num_points, MC_ERR_INVALID, "point id out of range");
        for (int i = 0; i < num_nodes; i++)
            for (int64_t k = c_off[i] + 1; k < c_off[i + 1]; k++)
                MC_REQUIRE(c_idx[k - 1] < c_idx[k], MC_ERR_INVALID, "contained ids must be ascending and unique per node");
        hipStream_t s = ctx->stream;
        ctx->have_graph = false;
        ctx->have_cluster = false;
        ctx->nodes_from_graph = false;
        ctx->F = num_frames;
        ctx->FW = (num_frames + 63) / 64;
        ctx->P = num_points;
        ctx->Mn = num_masks;
        ctx->N0 = num_nodes;
        ctx->nnzC0 = nc;
        ctx->n0_pts_total = np;
        const int n = num_nodes, FW = ctx->FW;
        ctx->d_n0_off.reserve((n + 1) * sizeof(int));
        ctx->d_n0_len.reserve((n + 1) * sizeof(int));
        ctx->d_n0_ptoff.reserve((n + 1) * sizeof(int));
        ctx->d_n0_ptlen.reserve((n + 1) * sizeof(int));
        ctx->d_n0_vf.reserve((static_cast<size_t>(n) * FW + 1) * 8);
        ctx->d_user_cidx.reserve((nc + 1) * sizeof(int));
        ctx->d_user_pts.reserve((np + 1) * sizeof(int));
        ctx->d_owner0.reserve((nc + 1) * sizeof(int));
        DevBuf t1, t2;
        t1.reserve((n + 1) * 8);
        t2.reserve((n + 1) * 8);
        if (n) {
            MC_HIP(hipMemcpyAsync(t1.ptr, c_off, (n + 1) * 8, hipMemcpyHostToDevice, s));
            MC_HIP(hipMemcpyAsync(t2.ptr, pt_off, (n + 1) * 8, hipMemcpyHostToDevice, s));
            if (FW) MC_HIP(hipMemcpyAsync(ctx->d_n0_vf.ptr, vf_bits, static_cast<size_t>(n) * FW * 8, hipMemcpyHostToDevice, s));
            if (nc) MC_HIP(hipMemcpyAsync(ctx->d_user_cidx.ptr, c_idx, nc * sizeof(int), hipMemcpyHostToDevice, s));
            if (np) MC_HIP(hipMemcpyAsync(ctx->d_user_pts.ptr, pt_idx, np * sizeof(int), hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_nodes_from_csr, grid_for(n), dim3(256), 0, s, n, t1.as<int64_t>(), t2.as<int64_t>(),
                               ctx->d_n0_off.as<int>(), ctx->d_n0_len.as<int>(), ctx->d_n0_ptoff.as<int>(),
                               ctx->d_n0_ptlen.as<int>(), ctx->d_owner0.as<int>());
        }
        MC_HIP(hipStreamSynchronize(s));
        t1.release();
        t2.release();
        ctx->n0_pool = ctx->d_user_cidx.as<int>();
        ctx->n0_pts = ctx->d_user_pts.as<int>();
        ctx->have_nodes = true;
    });
}

// ---------------------------------------------------------------------------------------------
// S6
// ---------------------------------------------------------------------------------------------
static mc::EdgeCap edge_cap(mc_ctx *ctx)
{
    if (ctx->cap_edges <= 0) return mc::EdgeCap{nullptr, nullptr, 0};
    return mc::EdgeCap{ctx->d_cap_buf.as<unsigned long long>(), ctx->d_cap_cnt.as<unsigned long long>(),
                       static_cast<long long>(ctx->cap_edges)};
}

// S6 iterations t_begin .. nthr-1 (after_pairs: iteration t_begin's pairs are done) and the final
// object state; the level-t node arrays are re-derived from the ping-pong pools
static void s6_iterations(mc_ctx *ctx, int t_begin, bool after_pairs)
{
    hipStream_t s = ctx->stream;
    const int nthr = ctx->s6_nthr, N0 = ctx->N0, FW = ctx->FW, Mn = ctx->Mn;
    const bool dense_obs = ctx->s6_dense_obs;
    const float ctf = ctx->s6_ctf;
    const size_t n0 = static_cast<size_t>(std::max(N0, 1));
    int *Nlev = ctx->d_Nlev.as<int>();
    int *dcap = ctx->d_cap.as<int>();
    MC_REQUIRE(t_begin == 0, MC_ERR_STATE, "S6 resumes only at iteration 0");
    const int *cur_off = ctx->d_n0_off.as<int>(), *cur_len = ctx->d_n0_len.as<int>(), *cur_pool = ctx->n0_pool;
    const unsigned long long *cur_vf = ctx->d_n0_vf.as<unsigned long long>();
    const dim3 gN = grid_for(N0), gW = grid_for(N0, mc::kPairWaves, 2048), gK = grid_for(N0, 1, 2048);
    for (int t = t_begin; t < nthr; t++) {
        const int *dN = Nlev + t;
        int *dNn = Nlev + t + 1;
        const bool toA = (t % 2) == 0;
        int *nx_off = toA ? ctx->d_offA.as<int>() : ctx->d_offB.as<int>();
        int *nx_len = toA ? ctx->d_lenA.as<int>() : ctx->d_lenB.as<int>();
        int *nx_pool = toA ? ctx->d_poolA.as<int>() : ctx->d_poolB.as<int>();
        int *nx_own = toA ? ctx->d_ownA.as<int>() : ctx->d_ownB.as<int>();
        unsigned long long *nx_vf = toA ? ctx->d_vfA.as<unsigned long long>() : ctx->d_vfB.as<unsigned long long>();
        if (t == t_begin && after_pairs) {
            // level 0's pairs ran on every rank's share and their forests were united
        } else if (!dense_obs) {
            TimedScope ts(ctx->timer, s, "s6_pairs");
            const mc::OvfWork ow{ctx->d_scratch.as<int>(), ctx->d_touched.as<int>(), N0, ctx->d_ovf_n.as<int>() + 1};
            hipLaunchKernelGGL(mc::k6_pairs, gW, dim3(256), 0, s, dN, cur_off, cur_len, cur_pool,
                               ctx->d_coloff.as<int>(), ctx->d_collen.as<int>(), ctx->d_colnodes.as<int>(), cur_vf, FW,
                               ctx->d_thr.as<float>(), t, ctf, ctx->d_parent.as<int>(),
                               ctx->d_edges.as<unsigned long long>(), ow, 0, 1, edge_cap(ctx));
        } else {
            TimedScope ts(ctx->timer, s, "s6_pairs");
            hipLaunchKernelGGL(mc::k6_parent_init, gN, dim3(256), 0, s, dN, ctx->d_parent.as<int>());
            hipLaunchKernelGGL(mc::k6_pairs_dense, dim3(4096), dim3(256), 0, s, dN, cur_vf, FW,
                               ctx->d_thr.as<float>(), t, ctx->d_parent.as<int>(),
                               ctx->d_edges.as<unsigned long long>(), edge_cap(ctx));
        }
        {
            TimedScope ts(ctx->timer, s, "s6_components");
            if (t > 0 && N0 <= kFusedComponentsMaxN0) {  // N_t <= N_1, typically N0 / 8: one workgroup
                hipLaunchKernelGGL(mc::k6_components, dim3(1), dim3(1024), 0, s, dN, dNn, ctx->d_parent.as<int>(),
                                   ctx->d_root.as<int>(), ctx->d_rank.as<int>(), cur_len, ctx->d_label.as<int>(),
                                   ctx->d_levels.as<int>() + static_cast<size_t>(t) * n0, ctx->d_memcnt.as<int>(),
                                   ctx->d_memoff.as<int>(), ctx->d_ublen.as<int>(), ctx->d_newoff.as<int>(),
                                   dcap + t + 1, ctx->d_members.as<int>(), ctx->d_ovf_n.as<int>());
            } else {
                hipLaunchKernelGGL(mc::k6_compress, gN, dim3(256), 0, s, dN, ctx->d_parent.as<int>(),
                                   ctx->d_root.as<int>(), ctx->d_isroot.as<int>(), ctx->d_ublen.as<int>(),
                                   ctx->d_ovf_n.as<int>());
                mc::scan_device_n(s, ctx->d_isroot.as<int>(), ctx->d_rank.as<int>(), dN, 0, dNn);
                hipLaunchKernelGGL(mc::k6_relabel, gN, dim3(256), 0, s, dN, ctx->d_root.as<int>(),
                                   ctx->d_rank.as<int>(), cur_len, ctx->d_label.as<int>(),
                                   ctx->d_levels.as<int>() + static_cast<size_t>(t) * n0, ctx->d_memcnt.as<int>(),
                                   ctx->d_ublen.as<int>());
                mc::scan_device_n(s, ctx->d_memcnt.as<int>(), ctx->d_memoff.as<int>(), dNn, 0, nullptr,
                                  ctx->d_ublen.as<int>(), ctx->d_newoff.as<int>(), dcap + t + 1);
                hipLaunchKernelGGL(mc::k6_memscatter, gN, dim3(256), 0, s, dN, 0, ctx->d_label.as<int>(),
                                   ctx->d_memoff.as<int>(), ctx->d_memcnt.as<int>(), ctx->d_members.as<int>(),
                                   nullptr);
            }
        }
        {
            TimedScope ts(ctx->timer, s, "s6_merge");
            // + the next iteration's column lists (nodes containing each mask, relabelled)
            const bool cols = !dense_obs && t + 1 < nthr;
            const mc::ColUpdate cu{Mn, dNn, ctx->d_coloff.as<int>(), ctx->d_collen.as<int>(),
                                   ctx->d_colnodes.as<int>(), cols ? ctx->d_label.as<int>() : nullptr,
                                   ctx->d_parent.as<int>(), N0, ctx->d_label.as<int>(),
                                   ctx->d_final_label.as<int>()};
            hipLaunchKernelGGL(mc::k6_merge, gK, dim3(256), 0, s, dNn, ctx->d_memoff.as<int>(),
                               ctx->d_members.as<int>(), cur_off, cur_len, cur_pool, cur_vf, FW,
                               ctx->d_newoff.as<int>(), nx_off, nx_len, nx_pool, nx_own, nx_vf, cu);
        }
        cur_off = nx_off;
        cur_len = nx_len;
        cur_pool = nx_pool;
        cur_vf = nx_vf;
    }
    ctx->fin_off = cur_off;
    ctx->fin_len = cur_len;
    ctx->fin_pool = cur_pool;
    ctx->fin_vf = cur_vf;
    ctx->n_iter = nthr;
    // ---- final point sets (node.py:35), per-object range bitmaps ----
    const int *dK = Nlev + nthr;
    int *stats = ctx->d_stats.as<int>();
    const bool point_path = ctx->nodes_from_graph;
    {
        TimedScope ts(ctx->timer, s, "s7_points");
        hipLaunchKernelGGL(mc::k7_reset, gN, dim3(256), 0, s, N0, ctx->d_pmin.as<int>(), ctx->d_pmax.as<int>());
        if (point_path) {
            hipLaunchKernelGGL(mc::k7_obj_of_mask, grid_for(ctx->M), dim3(256), 0, s, ctx->M,
                               ctx->d_node_of_mask.as<int>(), ctx->d_final_label.as<int>(),
                               ctx->d_obj_of_mask.as<int>());
            hipLaunchKernelGGL(mc::k7p_points<0>, dim3(ceil_div(ctx->P, 256)), dim3(256), 0, s, static_cast<int>(ctx->P),
                               ctx->d_pt_off.as<int>(), ctx->d_pt_list.as<unsigned>(), ctx->d_frame_start.as<int>(),
                               ctx->d_obj_of_mask.as<int>(), ctx->d_pmin.as<int>(), ctx->d_pmax.as<int>(), nullptr,
                               nullptr, stats + ST_OBJOVF);
        }
        else
            hipLaunchKernelGGL(mc::k7_minmax, gW, dim3(256), 0, s, N0, ctx->d_final_label.as<int>(),
                               ctx->d_n0_ptoff.as<int>(), ctx->d_n0_ptlen.as<int>(), ctx->n0_pts,
                               ctx->d_pmin.as<int>(), ctx->d_pmax.as<int>());
        hipLaunchKernelGGL(mc::k7_words, gN, dim3(256), 0, s, dK, ctx->d_pmin.as<int>(), ctx->d_pmax.as<int>(),
                           ctx->d_nwords.as<int>(), stats + ST_K);
        mc::scan_device_n(s, ctx->d_nwords.as<int>(), ctx->d_woff.as<int>(), dK, 0, stats + ST_WORDS);
    }
    sync_stats(ctx);  // bitmap capacity
    ctx->K = ctx->h_stats[ST_K];
    const bool use_points = point_path && ctx->h_stats[ST_OBJOVF] == 0;
    if (point_path && !use_points) {  // a point in > 8 objects: redo the ranges per node
        hipLaunchKernelGGL(mc::k7_reset, gN, dim3(256), 0, s, N0, ctx->d_pmin.as<int>(), ctx->d_pmax.as<int>());
        hipLaunchKernelGGL(mc::k7_minmax, gW, dim3(256), 0, s, N0, ctx->d_final_label.as<int>(),
                           ctx->d_n0_ptoff.as<int>(), ctx->d_n0_ptlen.as<int>(), ctx->n0_pts,
                           ctx->d_pmin.as<int>(), ctx->d_pmax.as<int>());
        hipLaunchKernelGGL(mc::k7_words, gN, dim3(256), 0, s, dK, ctx->d_pmin.as<int>(), ctx->d_pmax.as<int>(),
                           ctx->d_nwords.as<int>(), stats + ST_K);
        mc::scan_device_n(s, ctx->d_nwords.as<int>(), ctx->d_woff.as<int>(), dK, 0, stats + ST_WORDS);
        sync_stats(ctx);
    }
    const size_t words = static_cast<size_t>(std::max(ctx->h_stats[ST_WORDS], 1));
    ctx->d_bm.reserve(words * 8);
    {
        TimedScope ts(ctx->timer, s, "s7_points");
        MC_HIP(hipMemsetAsync(ctx->d_bm.ptr, 0, words * 8, s));
        if (use_points)
            hipLaunchKernelGGL(mc::k7p_points<1>, dim3(ceil_div(ctx->P, 256)), dim3(256), 0, s, static_cast<int>(ctx->P),
                               ctx->d_pt_off.as<int>(), ctx->d_pt_list.as<unsigned>(), ctx->d_frame_start.as<int>(),
                               ctx->d_obj_of_mask.as<int>(), ctx->d_pmin.as<int>(), ctx->d_pmax.as<int>(),
                               ctx->d_woff.as<int>(), ctx->d_bm.as<unsigned long long>(), stats + ST_OBJOVF);
        else
            hipLaunchKernelGGL(mc::k7_setbits, gW, dim3(256), 0, s, N0, ctx->d_final_label.as<int>(),
                               ctx->d_n0_ptoff.as<int>(), ctx->d_n0_ptlen.as<int>(), ctx->n0_pts,
                               ctx->d_pmin.as<int>(), ctx->d_woff.as<int>(), ctx->d_bm.as<unsigned long long>());
        hipLaunchKernelGGL(mc::k7_count, gK, dim3(256), 0, s, dK, ctx->d_woff.as<int>(),
                           ctx->d_bm.as<unsigned long long>(), ctx->d_ptcnt.as<int>());
        mc::scan_device_n(s, ctx->d_ptcnt.as<int>(), ctx->d_ptoff_out.as<int>(), dK, 0, stats + ST_NPTS);
        hipLaunchKernelGGL(mc::k7_extract, gK, dim3(256), 0, s, dK, ctx->d_woff.as<int>(),
                           ctx->d_bm.as<unsigned long long>(), ctx->d_pmin.as<int>(), ctx->d_ptoff_out.as<int>(),
                           ctx->d_pts_out.as<int>());
    }
    MC_HIP(hipGetLastError());
    MC_HIP(hipMemcpyAsync(ctx->h_stats, ctx->d_stats.ptr, ST_COUNT * sizeof(int), hipMemcpyDeviceToHost, s));
    ctx->have_cluster = true;
}

int mc_cluster_run(mc_ctx *ctx, const float *thresholds, int32_t n, double connect_threshold)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_nodes, MC_ERR_STATE, "mc_cluster_run before mc_graph_build / mc_nodes_set");
        // (edge capture on a sharded context: iteration 0 evaluates only this rank's pair rows, so its
        // capture holds those rows' edges and the driver gathers them, graph_shard.ShardedGraph.edges;
        // the later iterations run replicated and every rank captures all of their edges)
        hipStream_t s = ctx->stream;
        int *stats = ctx->d_stats.as<int>();
        if (ctx->nodes_from_graph) {
            sync_stats(ctx);  // the one host round trip between S4 and S6 (sizes for the S6 buffers)
            ctx->N0 = ctx->h_stats[ST_N0];
            ctx->nnzC0 = ctx->h_stats[ST_NNZC];
        }
        int nthr;
        if (thresholds) {
            MC_REQUIRE(n >= 0 && n <= 4096, MC_ERR_INVALID, "bad threshold count");
            nthr = n;
            ctx->d_thr.reserve((n + 1) * sizeof(float));
            if (n) MC_HIP(hipMemcpyAsync(ctx->d_thr.ptr, thresholds, n * sizeof(float), hipMemcpyHostToDevice, s));
        } else {
            MC_REQUIRE(ctx->nodes_from_graph, MC_ERR_STATE, "device thresholds need mc_graph_build");
            if (ctx->h_stats[ST_THR_STATUS] != MC_OK)
                throw McError{ctx->h_stats[ST_THR_STATUS], "no positive observer count (np.percentile of an empty array)"};
            nthr = ctx->h_stats[ST_NTHR];
        }
        const int N0 = ctx->N0, FW = ctx->FW, Mn = ctx->Mn;
        MC_REQUIRE(!(N0 == 0 && nthr > 0), MC_ERR_NO_NODES, "no nodes to cluster (torch.stack of an empty list)");
        const bool dense = !(connect_threshold > 0.0);  // ct <= 0: all pairs with O >= thr (NaN: no edge)
        const bool ct_nan = std::isnan(connect_threshold);
        const bool dense_obs = dense && !ct_nan;
        const float ctf = static_cast<float>(connect_threshold);  // torch compares in float32
        const size_t n0 = static_cast<size_t>(std::max(N0, 1));
        const size_t cap = static_cast<size_t>(std::max<int64_t>(ctx->nnzC0, 1));
        ctx->d_parent.reserve(n0 * 4);
        ctx->d_root.reserve(n0 * 4);
        ctx->d_isroot.reserve(n0 * 4);
        ctx->d_rank.reserve((n0 + 1) * 4);
        ctx->d_label.reserve(n0 * 4);
        ctx->d_levels.reserve(std::max<size_t>(1, static_cast<size_t>(nthr)) * n0 * 4);
        const bool fresh_memcnt = ctx->d_memcnt.bytes < n0 * 4;
        ctx->d_memcnt.reserve(n0 * 4);
        if (fresh_memcnt) MC_HIP(hipMemsetAsync(ctx->d_memcnt.ptr, 0, ctx->d_memcnt.bytes, s));  // kept zero by K9
        ctx->d_memoff.reserve((n0 + 1) * 4);
        ctx->d_ublen.reserve(n0 * 4);
        ctx->d_newoff.reserve((n0 + 1) * 4);
        ctx->d_members.reserve(n0 * 4);
        const bool fresh_colcnt = ctx->d_colcnt.bytes < static_cast<size_t>(Mn + 1) * 4;
        ctx->d_colcnt.reserve((Mn + 1) * 4);
        if (fresh_colcnt) MC_HIP(hipMemsetAsync(ctx->d_colcnt.ptr, 0, ctx->d_colcnt.bytes, s));  // kept zero by K3
        ctx->d_coloff.reserve((Mn + 2) * 4);
        ctx->d_collen.reserve((Mn + 1) * 4);
        ctx->d_colnodes.reserve(cap * 4);
        if (!ctx->d_ovf_n.ptr) {
            ctx->d_ovf_n.reserve((1 + mc::kOvfSlots) * 4);  // [0] unused counter (K5 clears it), [1..] slot locks
            MC_HIP(hipMemsetAsync(ctx->d_ovf_n.ptr, 0, (1 + mc::kOvfSlots) * 4, s));  // locks kept zero
        }
        constexpr int kOvfBlocks = mc::kOvfSlots;
        if (ctx->scratch_n0 < N0) {
            ctx->d_scratch.reserve(static_cast<size_t>(kOvfBlocks) * n0 * 4);
            ctx->d_touched.reserve(static_cast<size_t>(kOvfBlocks) * n0 * 4);
            MC_HIP(hipMemsetAsync(ctx->d_scratch.ptr, 0, static_cast<size_t>(kOvfBlocks) * n0 * 4, s));
            ctx->scratch_n0 = N0;
        }
        ctx->d_edges.reserve(static_cast<size_t>(std::max(nthr, 1)) * mc::kSpread * mc::kSpreadStrideL * 8);  // spread slots
        ctx->d_Nlev.reserve((nthr + 2) * 4);
        ctx->d_cap.reserve((nthr + 2) * 4);
        ctx->d_final_label.reserve(n0 * 4);
        ctx->d_poolA.reserve(cap * 4);
        ctx->d_poolB.reserve(cap * 4);
        ctx->d_ownA.reserve(cap * 4);
        ctx->d_ownB.reserve(cap * 4);
        ctx->d_offA.reserve(n0 * 4);
        ctx->d_offB.reserve(n0 * 4);
        ctx->d_lenA.reserve(n0 * 4);
        ctx->d_lenB.reserve(n0 * 4);
        ctx->d_vfA.reserve(n0 * FW * 8 + 8);
        ctx->d_vfB.reserve(n0 * FW * 8 + 8);
        ctx->d_pmin.reserve(n0 * 4);
        ctx->d_pmax.reserve(n0 * 4);
        ctx->d_nwords.reserve(n0 * 4);
        ctx->d_woff.reserve((n0 + 1) * 4);
        ctx->d_ptcnt.reserve(n0 * 4);
        ctx->d_ptoff_out.reserve((n0 + 1) * 4);
        ctx->d_pts_out.reserve((ctx->n0_pts_total + 1) * 4);

        int *Nlev = ctx->d_Nlev.as<int>();
        int *dcap = ctx->d_cap.as<int>();
        hipLaunchKernelGGL(mc::k6_init, grid_for(std::max<int64_t>(N0, nthr)), dim3(256), 0, s, N0,
                           ctx->d_final_label.as<int>(), ctx->nodes_from_graph ? stats + ST_N0 : nullptr, N0, Nlev,
                           dcap, ctx->nodes_from_graph ? stats + ST_NNZC : nullptr, static_cast<int>(ctx->nnzC0),
                           ctx->d_edges.as<unsigned long long>(), nthr);

        if (ctx->cap_edges > 0) {
            ctx->d_cap_buf.reserve(static_cast<size_t>(ctx->cap_edges) * 8);
            ctx->d_cap_cnt.reserve(8);
            MC_HIP(hipMemsetAsync(ctx->d_cap_cnt.ptr, 0, 8, s));
        }
        const dim3 gE = grid_for(std::max<int64_t>(N0, ctx->nnzC0)), gC = grid_for(std::max(N0, Mn), 64, 8192);
        const int *cur_pool = ctx->n0_pool, *cur_own = ctx->d_owner0.as<int>();
        if (!dense_obs && nthr > 0) {  // level-0 column lists (nodes contained by each mask)
            TimedScope ts(ctx->timer, s, "s6_columns");
            hipLaunchKernelGGL(mc::k6_colcount, gE, dim3(256), 0, s, Nlev, dcap, cur_pool, cur_own,
                               ctx->d_parent.as<int>(), ctx->d_colcnt.as<int>());
            mc::scan_device_n(s, ctx->d_colcnt.as<int>(), ctx->d_coloff.as<int>(), nullptr, Mn, nullptr);
            hipLaunchKernelGGL(mc::k6_colscatter, gE, dim3(256), 0, s, dcap, cur_pool, cur_own,
                               ctx->d_coloff.as<int>(), ctx->d_colcnt.as<int>(), ctx->d_colnodes.as<int>());
            hipLaunchKernelGGL(mc::k6_colupdate, gC, dim3(64), 0, s, Mn, Nlev, ctx->d_coloff.as<int>(),
                               ctx->d_collen.as<int>(), ctx->d_colnodes.as<int>(), nullptr, ctx->d_parent.as<int>());
        }
        ctx->s6_nthr = nthr;
        ctx->s6_dense_obs = dense_obs;
        ctx->s6_ctf = ctf;
        ctx->have_cluster = false;
        ctx->sh_pending = 0;
        if (nthr > 0 && N0 > 0 && sharded(ctx) && !dense_obs) {
            // iteration 0 (the N0 x N0 pairs) on this rank's rows; the union-find forests of all
            // ranks are united by mc_shard_import(MC_SHARD_FOREST), which runs the rest
            TimedScope ts(ctx->timer, s, "s6_pairs");
            const mc::OvfWork ow{ctx->d_scratch.as<int>(), ctx->d_touched.as<int>(), N0, ctx->d_ovf_n.as<int>() + 1};
            hipLaunchKernelGGL(mc::k6_pairs, grid_for(N0, mc::kPairWaves, 2048), dim3(256), 0, s, Nlev,
                               ctx->d_n0_off.as<int>(), ctx->d_n0_len.as<int>(), ctx->n0_pool, ctx->d_coloff.as<int>(),
                               ctx->d_collen.as<int>(), ctx->d_colnodes.as<int>(), ctx->d_n0_vf.as<unsigned long long>(),
                               FW, ctx->d_thr.as<float>(), 0, ctf, ctx->d_parent.as<int>(),
                               ctx->d_edges.as<unsigned long long>(), ow, ctx->sh_rank, ctx->sh_world,
                               mc::EdgeCap{nullptr, nullptr, 0});
            MC_HIP(hipGetLastError());
            ctx->sh_pending = MC_SHARD_FOREST;
            if (ctx->comm) shard_drain_native(ctx);  // the forests over RCCL, then the rest of S6
            return;
        }
        s6_iterations(ctx, 0, false);
    });
}

// ---------------------------------------------------------------------------------------------
// row-block sharding over processes; kernels in mc_shard_kernels.inl
// ---------------------------------------------------------------------------------------------
int mc_shard_set(mc_ctx *ctx, int32_t rank, int32_t world)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(world >= 1 && world <= 1024 && rank >= 0 && rank < world, MC_ERR_INVALID, "bad rank / world");
        MC_REQUIRE(!ctx->comm, MC_ERR_STATE, "a communicator is attached (rank / world come from it; detach first)");
        ctx->sh_rank = rank;
        ctx->sh_world = world;
        ctx->sh_pending = 0;
        if (ctx->have_scene) build_s3_lists(ctx, frame_starts(ctx));
    });
}

int mc_shard_pending(mc_ctx *ctx, int32_t *phase)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(phase, MC_ERR_INVALID, "null phase");
        *phase = ctx->sh_pending;
    });
}

static void shard_export(mc_ctx *ctx, int32_t phase, void *dst_dev, int64_t *bytes)
{
    {
        MC_REQUIRE(bytes, MC_ERR_INVALID, "null bytes");
        MC_REQUIRE(phase == ctx->sh_pending && phase != 0, MC_ERR_STATE, "no such exchange pending");
        hipStream_t s = ctx->stream;
        if (phase == MC_SHARD_S3) {
            const int nr = ctx->sh_r1 - ctx->sh_r0;
            if (ctx->sh_s3_words < 0) {  // entry offsets of this rank's rows + their total (one host sync)
                ctx->d_sh_eoff.reserve((nr + 2) * 4);
                DevBuf dt;
                dt.reserve(8);
                mc::scan_device_n(s, ctx->d_crow_len.as<int>() + ctx->sh_r0, ctx->d_sh_eoff.as<int>(), nullptr, nr,
                                  dt.as<int>());
                int h = 0;
                MC_HIP(hipMemcpyAsync(&h, dt.ptr, 4, hipMemcpyDeviceToHost, s));
                MC_HIP(hipStreamSynchronize(s));
                ctx->sh_s3_words = 2 + 2 * static_cast<int64_t>(nr) + h;
            }
            *bytes = 4 * ctx->sh_s3_words;
            if (dst_dev)
                hipLaunchKernelGGL(mc::k_sh_s3_pack, grid_for(std::max(nr, 1) * 64, 256, 2048), dim3(256), 0, s,
                                   ctx->sh_r0, ctx->sh_r1, ctx->F, ctx->d_ctmp.as<int>(), ctx->d_crow_len.as<int>(),
                                   ctx->d_useg.as<unsigned char>(), ctx->d_sh_eoff.as<int>(), static_cast<int *>(dst_dev));
        } else if (phase == MC_SHARD_HIST) {
            *bytes = 8 * static_cast<int64_t>(ctx->F + 1);
            if (dst_dev)
                MC_HIP(hipMemcpyAsync(dst_dev, ctx->d_hist.ptr, *bytes, hipMemcpyDeviceToDevice, s));
        } else if (phase == MC_SHARD_FOREST) {
            *bytes = 4 * (static_cast<int64_t>(ctx->N0) + 2);
            if (dst_dev)
                hipLaunchKernelGGL(mc::k_sh_forest_export, grid_for(ctx->N0), dim3(256), 0, s, ctx->d_Nlev.as<int>(),
                                   ctx->d_parent.as<int>(), ctx->d_edges.as<unsigned long long>(),
                                   static_cast<int *>(dst_dev), ctx->N0);
        } else {
            throw McError{MC_ERR_INVALID, "unknown exchange phase"};
        }
        MC_HIP(hipGetLastError());
    }
}

static void shard_import(mc_ctx *ctx, int32_t phase, const void *src_dev, int64_t stride_bytes)
{
    {
        MC_REQUIRE(phase == ctx->sh_pending && phase != 0, MC_ERR_STATE, "no such exchange pending");
        MC_REQUIRE(src_dev, MC_ERR_INVALID, "null source");
        hipStream_t s = ctx->stream;
        const int W = ctx->sh_world;
        if (phase == MC_SHARD_S3) {
            MC_REQUIRE(stride_bytes % 4 == 0 && stride_bytes >= 8, MC_ERR_INVALID, "bad S3 block stride");
            hipLaunchKernelGGL(mc::k_sh_s3_unpack, dim3(mc::kUnpackWg, W), dim3(256), 0, s,
                               static_cast<const int *>(src_dev), static_cast<long long>(stride_bytes / 4), ctx->sh_rank,
                               ctx->F, ctx->d_ctmp.as<int>(), ctx->d_crow_len.as<int>(), ctx->d_useg.as<unsigned char>());
            MC_HIP(hipGetLastError());
            ctx->sh_pending = MC_SHARD_HIST;
            graph_build_tail(ctx);  // undo + S5 replicated, this rank's S4 tiles
        } else if (phase == MC_SHARD_HIST) {
            // src: the histogram summed over the ranks
            MC_HIP(hipMemcpyAsync(ctx->d_hist.ptr, src_dev, 8 * static_cast<size_t>(ctx->F + 1), hipMemcpyDeviceToDevice, s));
            ctx->sh_pending = 0;
            graph_build_thresholds(ctx);
        } else if (phase == MC_SHARD_FOREST) {
            MC_REQUIRE(stride_bytes % 4 == 0 && stride_bytes >= 4 * (static_cast<int64_t>(ctx->N0) + 2), MC_ERR_INVALID,
                       "bad FOREST block stride");
            {
                TimedScope ts(ctx->timer, s, "s6_pairs");
                hipLaunchKernelGGL(mc::k_sh_forest_import, dim3(grid_for(ctx->N0, 256, 1024).x, W), dim3(256), 0, s,
                                   ctx->d_Nlev.as<int>(), static_cast<const int *>(src_dev),
                                   static_cast<long long>(stride_bytes / 4), ctx->sh_rank, ctx->N0,
                                   ctx->d_parent.as<int>(), ctx->d_edges.as<unsigned long long>());
            }
            MC_HIP(hipGetLastError());
            ctx->sh_pending = 0;
            s6_iterations(ctx, 0, true);
        } else {
            throw McError{MC_ERR_INVALID, "unknown exchange phase"};
        }
    }
}

int mc_shard_export(mc_ctx *ctx, int32_t phase, void *dst_dev, int64_t *bytes)
{
    return guarded(ctx, [&] { shard_export(ctx, phase, dst_dev, bytes); });
}

int mc_shard_import(mc_ctx *ctx, int32_t phase, const void *src_dev, int64_t stride_bytes)
{
    return guarded(ctx, [&] { shard_import(ctx, phase, src_dev, stride_bytes); });
}

// ---- native collectives: RCCL, loaded on first use ------------------------------------------
namespace {
struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclCommCount) comm_count = nullptr;
    decltype(&ncclCommUserRank) comm_user_rank = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl *rccl_lib()
{
    static const Rccl r = [] {
        Rccl x;
        void *h = nullptr;
        for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) return x;
        x.get_unique_id = reinterpret_cast<decltype(x.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
        x.comm_init_rank = reinterpret_cast<decltype(x.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
        x.comm_destroy = reinterpret_cast<decltype(x.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        x.comm_count = reinterpret_cast<decltype(x.comm_count)>(dlsym(h, "ncclCommCount"));
        x.comm_user_rank = reinterpret_cast<decltype(x.comm_user_rank)>(dlsym(h, "ncclCommUserRank"));
        x.all_reduce = reinterpret_cast<decltype(x.all_reduce)>(dlsym(h, "ncclAllReduce"));
        x.all_gather = reinterpret_cast<decltype(x.all_gather)>(dlsym(h, "ncclAllGather"));
        x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(h, "ncclGetErrorString"));
        return x;
    }();
    MC_REQUIRE(r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.comm_count && r.comm_user_rank &&
                   r.all_reduce && r.all_gather && r.error_string,
               MC_ERR_UNSUPPORTED, "RCCL (librccl.so.1) not loadable");
    return &r;
}

void rccl_check(ncclResult_t e, const char *what)
{
    if (e != ncclSuccess) throw McError{MC_ERR_HIP, std::string(what) + ": " + rccl_lib()->error_string(e)};
}

bool sharded(const mc_ctx *ctx) { return ctx->sh_world > 1 || ctx->comm; }
}  // namespace

// every pending exchange over the attached communicator, stream-ordered on the context stream:
// the S3 and FOREST blocks all-gathered into [world][stride] (S3's stride from a max all-reduce of
// the block sizes, one host read), the HIST block all-reduced (sum, int64)
static void shard_drain_native(mc_ctx *ctx)
{
    const Rccl &r = *rccl_lib();
    hipStream_t s = ctx->stream;
    auto comm = static_cast<ncclComm_t>(ctx->comm);
    const size_t W = static_cast<size_t>(ctx->sh_world);
    while (ctx->sh_pending) {
        const int ph = ctx->sh_pending;
        int64_t bytes = 0;
        shard_export(ctx, ph, nullptr, &bytes);
        if (ph == MC_SHARD_HIST) {
            const size_t n = static_cast<size_t>(bytes) / 8;
            ctx->d_sh_send.reserve(n * 8);
            ctx->d_sh_recv.reserve(n * 8);
            shard_export(ctx, ph, ctx->d_sh_send.ptr, &bytes);
            rccl_check(r.all_reduce(ctx->d_sh_send.ptr, ctx->d_sh_recv.ptr, n, ncclInt64, ncclSum, comm, s),
                       "ncclAllReduce (observer histogram)");
            shard_import(ctx, ph, ctx->d_sh_recv.ptr, 0);
            continue;
        }
        int64_t n_max = bytes;
        if (ph == MC_SHARD_S3) {
            ctx->d_sh_size.reserve(8);
            MC_HIP(hipMemcpy(ctx->d_sh_size.ptr, &bytes, 8, hipMemcpyHostToDevice));  // done at return
            rccl_check(r.all_reduce(ctx->d_sh_size.ptr, ctx->d_sh_size.ptr, 1, ncclInt64, ncclMax, comm, s),
                       "ncclAllReduce (S3 block size)");
            MC_HIP(hipMemcpyAsync(&n_max, ctx->d_sh_size.ptr, 8, hipMemcpyDeviceToHost, s));
            MC_HIP(hipStreamSynchronize(s));
        }
        const size_t words = static_cast<size_t>(std::max<int64_t>((n_max + 3) / 4, 1));
        ctx->d_sh_send.reserve(words * 4);
        ctx->d_sh_recv.reserve(W * words * 4);
        MC_HIP(hipMemsetAsync(ctx->d_sh_send.ptr, 0, words * 4, s));
        shard_export(ctx, ph, ctx->d_sh_send.ptr, &bytes);
        rccl_check(r.all_gather(ctx->d_sh_send.ptr, ctx->d_sh_recv.ptr, words, ncclInt32, comm, s),
                   ph == MC_SHARD_S3 ? "ncclAllGather (S3 rows)" : "ncclAllGather (union-find forests)");
        shard_import(ctx, ph, ctx->d_sh_recv.ptr, static_cast<int64_t>(4 * words));
    }
}

static void comm_detach(mc_ctx *ctx)
{
    if (ctx->comm && ctx->own_comm) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)rccl_lib()->comm_destroy(static_cast<ncclComm_t>(ctx->comm));
    }
    ctx->comm = nullptr;
    ctx->own_comm = false;
}

static void comm_attach(mc_ctx *ctx, void *comm, bool own)
{
    int rank = 0, world = 1;
    rccl_check(rccl_lib()->comm_user_rank(static_cast<ncclComm_t>(comm), &rank), "ncclCommUserRank");
    rccl_check(rccl_lib()->comm_count(static_cast<ncclComm_t>(comm), &world), "ncclCommCount");
    comm_detach(ctx);
    ctx->comm = comm;
    ctx->own_comm = own;
    ctx->sh_rank = rank;
    ctx->sh_world = world;
    ctx->sh_pending = 0;
    if (ctx->have_scene) build_s3_lists(ctx, frame_starts(ctx));
}

int mc_comm_unique_id(uint8_t id[MC_COMM_ID_BYTES])
{
    static_assert(MC_COMM_ID_BYTES == sizeof(ncclUniqueId), "unique id size");
    if (!id) return MC_ERR_INVALID;
    try {
        ncclUniqueId u;
        rccl_check(rccl_lib()->get_unique_id(&u), "ncclGetUniqueId");
        memcpy(id, &u, sizeof(u));
        return MC_OK;
    } catch (const McError &e) {
        return e.code;
    }
}

int mc_ctx_comm_init(mc_ctx *ctx, const uint8_t id[MC_COMM_ID_BYTES], int32_t rank, int32_t world)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(id, MC_ERR_INVALID, "null unique id");
        MC_REQUIRE(world >= 1 && world <= 1024 && rank >= 0 && rank < world, MC_ERR_INVALID, "bad rank / world");
        MC_HIP(hipSetDevice(ctx->device));
        ncclUniqueId u;
        memcpy(&u, id, sizeof(u));
        ncclComm_t c = nullptr;
        rccl_check(rccl_lib()->comm_init_rank(&c, world, u, rank), "ncclCommInitRank");
        comm_attach(ctx, c, true);
    });
}

int mc_ctx_attach_comm(mc_ctx *ctx, void *nccl_comm)
{
    return guarded(ctx, [&] {
        if (!nccl_comm) {
            comm_detach(ctx);
            ctx->sh_rank = 0;
            ctx->sh_world = 1;
            ctx->sh_pending = 0;
            if (ctx->have_scene) build_s3_lists(ctx, frame_starts(ctx));
            return;
        }
        comm_attach(ctx, nccl_comm, false);
    });
}

int mc_cluster_set_edge_capture(mc_ctx *ctx, int64_t capacity)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(capacity >= 0, MC_ERR_INVALID, "negative capacity");
        ctx->cap_edges = capacity;
    });
}

int mc_cluster_get_edges(mc_ctx *ctx, uint64_t *keys, int64_t *n)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_cluster && n, MC_ERR_STATE, "no clustering result");
        MC_REQUIRE(ctx->cap_edges > 0, MC_ERR_STATE, "edge capture is off");
        unsigned long long cnt = 0;
        MC_HIP(hipMemcpyAsync(&cnt, ctx->d_cap_cnt.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
        *n = static_cast<int64_t>(cnt);
        if (keys && cnt) {
            MC_REQUIRE(static_cast<int64_t>(cnt) <= ctx->cap_edges, MC_ERR_UNSUPPORTED,
                       "more edges than the capture capacity (raise it and run again)");
            MC_HIP(hipMemcpyAsync(keys, ctx->d_cap_buf.ptr, cnt * 8, hipMemcpyDeviceToHost, ctx->stream));
            MC_HIP(hipStreamSynchronize(ctx->stream));
        }
    });
}

int mc_cluster_get_info(mc_ctx *ctx, mc_cluster_info *info)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_cluster && info, MC_ERR_STATE, "no clustering result");
        sync_stats(ctx);
        info->num_iterations = ctx->n_iter;
        info->num_objects = ctx->h_stats[ST_K];
        info->num_nodes0 = ctx->N0;
        info->reserved = 0;
        info->num_object_points = ctx->h_stats[ST_NPTS];
        std::vector<int> len(std::max(ctx->K, 1));
        if (ctx->K) MC_HIP(hipMemcpyAsync(len.data(), ctx->fin_len, ctx->K * 4, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
        int64_t tot = 0;
        for (int k = 0; k < ctx->K; k++) tot += len[k];
        info->num_object_contained = tot;
        info->num_object_masks = ctx->N0;
    });
}

int mc_cluster_get_level_sizes(mc_ctx *ctx, int32_t *sizes)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_cluster, MC_ERR_STATE, "no clustering result");
        MC_HIP(hipMemcpyAsync(sizes, ctx->d_Nlev.ptr, (ctx->n_iter + 1) * 4, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int mc_cluster_get_level_caps(mc_ctx *ctx, int32_t *caps)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_cluster, MC_ERR_STATE, "no clustering result");
        MC_HIP(hipMemcpyAsync(caps, ctx->d_cap.ptr, (ctx->n_iter + 1) * 4, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int mc_cluster_get_partition(mc_ctx *ctx, int32_t iteration, int32_t *labels)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_cluster, MC_ERR_STATE, "no clustering result");
        MC_REQUIRE(iteration >= 0 && iteration < ctx->n_iter, MC_ERR_INVALID, "iteration out of range");
        int nt = 0;
        MC_HIP(hipMemcpyAsync(&nt, ctx->d_Nlev.as<int>() + iteration, 4, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
        const size_t n0 = static_cast<size_t>(std::max(ctx->N0, 1));
        if (nt)
            MC_HIP(hipMemcpyAsync(labels, ctx->d_levels.as<int>() + static_cast<size_t>(iteration) * n0, nt * 4,
                                  hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int mc_cluster_get_edge_counts(mc_ctx *ctx, int64_t *edges)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_cluster, MC_ERR_STATE, "no clustering result");
        const size_t per = static_cast<size_t>(mc::kSpread) * mc::kSpreadStrideL;
        std::vector<unsigned long long> h(static_cast<size_t>(ctx->n_iter) * per);
        if (ctx->n_iter)
            MC_HIP(hipMemcpyAsync(h.data(), ctx->d_edges.ptr, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
        for (int t = 0; t < ctx->n_iter; t++) {  // fold the spread slots
            unsigned long long v = 0;
            for (int k = 0; k < mc::kSpread; k++) v += h[t * per + k * mc::kSpreadStrideL];
            edges[t] = static_cast<int64_t>(v);
        }
    });
}

int mc_cluster_get_final_labels(mc_ctx *ctx, int32_t *labels)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_cluster, MC_ERR_STATE, "no clustering result");
        if (ctx->N0) MC_HIP(hipMemcpyAsync(labels, ctx->d_final_label.ptr, ctx->N0 * 4, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int mc_cluster_get_objects(mc_ctx *ctx, uint64_t *vf_bits, int64_t *c_off, int32_t *c_idx, int64_t *pt_off,
                           int32_t *pt_idx, int64_t *mask_off, int32_t *mask_idx)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_cluster, MC_ERR_STATE, "no clustering result");
        sync_stats(ctx);
        const int K = ctx->K, FW = ctx->FW;
        hipStream_t s = ctx->stream;
        std::vector<int> off(std::max(K, 1)), len(std::max(K, 1)), poff(K + 1);
        if (K) {
            MC_HIP(hipMemcpyAsync(off.data(), ctx->fin_off, K * 4, hipMemcpyDeviceToHost, s));
            MC_HIP(hipMemcpyAsync(len.data(), ctx->fin_len, K * 4, hipMemcpyDeviceToHost, s));
            MC_HIP(hipMemcpyAsync(poff.data(), ctx->d_ptoff_out.ptr, (K + 1) * 4, hipMemcpyDeviceToHost, s));
            if (vf_bits && FW) MC_HIP(hipMemcpyAsync(vf_bits, ctx->fin_vf, static_cast<size_t>(K) * FW * 8, hipMemcpyDeviceToHost, s));
        }
        MC_HIP(hipStreamSynchronize(s));
        if (c_off) {
            c_off[0] = 0;
            int64_t end = 0;
            for (int k = 0; k < K; k++) {
                c_off[k + 1] = c_off[k] + len[k];
                if (len[k]) end = std::max<int64_t>(end, static_cast<int64_t>(off[k]) + len[k]);
            }
            if (c_idx && end) {  // one copy of the pool span, rows gathered on the host
                std::vector<int> pool(end);
                MC_HIP(hipMemcpyAsync(pool.data(), ctx->fin_pool, end * 4, hipMemcpyDeviceToHost, s));
                MC_HIP(hipStreamSynchronize(s));
                for (int k = 0; k < K; k++)
                    if (len[k]) memcpy(c_idx + c_off[k], pool.data() + off[k], static_cast<size_t>(len[k]) * 4);
            }
        }
        if (pt_off) {
            for (int k = 0; k <= K; k++) pt_off[k] = K ? poff[k] : 0;
            const int np = K ? poff[K] : 0;
            if (pt_idx && np) MC_HIP(hipMemcpyAsync(pt_idx, ctx->d_pts_out.ptr, static_cast<size_t>(np) * 4, hipMemcpyDeviceToHost, s));
        }
        MC_HIP(hipStreamSynchronize(s));
        if (mask_off) {
            // members of each object as ascending level-0 node ids (stable counting sort)
            std::vector<int> fl(std::max(ctx->N0, 1));
            if (ctx->N0) MC_HIP(hipMemcpy(fl.data(), ctx->d_final_label.ptr, ctx->N0 * 4, hipMemcpyDeviceToHost));
            std::vector<int64_t> cnt(K + 1, 0);
            for (int i = 0; i < ctx->N0; i++) cnt[fl[i] + 1]++;
            for (int k = 0; k < K; k++) cnt[k + 1] += cnt[k];
            for (int k = 0; k <= K; k++) mask_off[k] = cnt[k];
            if (mask_idx)
                for (int i = 0; i < ctx->N0; i++) mask_idx[cnt[fl[i]]++] = i;
        }
    });
}

// ---------------------------------------------------------------------------------------------
// S1 back-projection
// ---------------------------------------------------------------------------------------------
__global__ void k_fill_u32(unsigned *p, size_t n, unsigned v)
{
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256) p[i] = v;
}

}  // extern "C"

namespace {

void fill_u32(hipStream_t s, void *p, size_t n, unsigned v)
{
    if (n) hipLaunchKernelGGL(k_fill_u32, grid_for(static_cast<int64_t>(n)), dim3(256), 0, s, static_cast<unsigned *>(p), n, v);
}

// grow a device buffer, keeping its first `used` bytes
void grow_keep(DevBuf &b, size_t bytes, size_t used, hipStream_t s)
{
    if (bytes <= b.bytes) return;
    DevBuf nb;
    nb.reserve(bytes + bytes / 2);
    if (used) MC_HIP(hipMemcpyAsync(nb.ptr, b.ptr, used, hipMemcpyDeviceToDevice, s));
    MC_HIP(hipStreamSynchronize(s));
    b.swap(nb);  // the old buffer is freed with nb
}

enum BpStat : int {
    BS_ERRF = 0, BS_VOXERR, BS_OVF, BS_TOP, BS_NS, BS_NPX, BS_M, BS_NNZ,
    BS_CLS,             // denoise size-class counts (kBpClasses LDS classes + the global-memory kernel)
    BS_TK = BS_CLS + mc::kBpClasses + 1,  // ticket counters of the LDS classes
    BS_VXFB = BS_TK + mc::kBpClasses,     // slots the first voxel tier hands to the second
    BS_VXFB2,                             // slots the second voxel tier hands to k_bp_voxel
    BS_DQ,                                // points queued for the k-NN ring search
    BS_DNERR,                             // denoise internal-error bits (queue entry / region out of range)
    BS_PXOVF,                             // the batch's mask pixels exceed the capacity: grown, batch redone
    BS_COUNT
};

size_t slots_cap(int fb) { return static_cast<size_t>(fb) * 256 + 1; }  // (frame, id) slots of a batch
// HBM of the per-batch S1 arrays (bp_reserve): per mask pixel (the arrays indexed by pixel-list position,
// voxel and point arrays included: 195 B) and per frame pixel (the valid-id map); the per-slot and
// per-frame ones are small against them.  A batch's frames are sized for its mask pixels: the share of
// mask pixels among frame pixels seen so far (bp_mfrac, 1 before any batch) decides the frames per batch,
// and a batch with more mask pixels than its capacity grows the arrays and is redone.
constexpr size_t kBpBytesPerMaskPixel = 196;
constexpr size_t kBpBytesPerFramePixel = 2;

// (re)allocate the per-batch arrays for fb frames of H x W (pixel capacity fb*H*W)
// Workgroups per resident slot of a denoise class (the classes take slots from tickets): the extra
// ones start on CUs that other classes free, so no class keeps only its initial share of the chip.
#ifndef MC_BP_OVERSUB
#define MC_BP_OVERSUB 2
#endif
constexpr int kBpOversub = MC_BP_OVERSUB;  // class grids: resident workgroups x this (slots come from tickets)
// u16 entries of per-workgroup eps-neighbour lists before class cls's region
inline size_t nbl_offset(const mc_ctx *ctx, int cls)
{
    const size_t per_cls[mc::kBpClasses] = {static_cast<size_t>(mc::BpLdsClass<512>::kWgPerCu) * 512,
                                            static_cast<size_t>(mc::BpLdsClass<1024>::kWgPerCu) * 1024,
                                            static_cast<size_t>(mc::BpLdsClass<2048>::kWgPerCu) * 2048,
                                            static_cast<size_t>(mc::BpLdsClass<3072>::kWgPerCu) * 3072,
                                            static_cast<size_t>(mc::BpLdsClass<4096>::kWgPerCu) * 4096,
                                            static_cast<size_t>(mc::BpLdsClass<16384>::kWgPerCu) * 16384};
    size_t o = 0;
    for (int c = 0; c < cls; c++) o += per_cls[c];
    return o * static_cast<size_t>(ctx->num_cu) * kBpOversub * mc::kBpNbCap;
}

// ints of per-workgroup lean scratch before class cls's region
inline size_t lean_offset(const mc_ctx *ctx, int cls)
{
    const size_t per_cls[mc::kBpClasses] = {
        mc::kBpLeanInts<512> * mc::BpLdsClass<512>::kWgPerCu, mc::kBpLeanInts<1024> * mc::BpLdsClass<1024>::kWgPerCu,
        mc::kBpLeanInts<2048> * mc::BpLdsClass<2048>::kWgPerCu, mc::kBpLeanInts<3072> * mc::BpLdsClass<3072>::kWgPerCu,
        mc::kBpLeanInts<4096> * mc::BpLdsClass<4096>::kWgPerCu,
        mc::kBpLeanInts<16384> * mc::BpLdsClass<16384>::kWgPerCu};
    size_t o = 0;
    for (int c = 0; c < cls; c++) o += per_cls[c];
    return o * static_cast<size_t>(ctx->num_cu) * kBpOversub;
}

void bp_reserve(mc_ctx *ctx, int fb, int H, int W, int nbands, size_t mask_px, hipStream_t s)
{
    const size_t px = mask_px + 1;
    const size_t slots = slots_cap(fb);
    ctx->d_band.reserve(static_cast<size_t>(fb) * nbands * mc::kBpWaves * 256 * 4);
    ctx->d_bpvid.reserve(static_cast<size_t>(fb) * H * W + 16);
    ctx->bp_fpx_cap = std::max(ctx->bp_fpx_cap, static_cast<size_t>(fb) * H * W);
    ctx->d_present.reserve(static_cast<size_t>(fb) * 8 * 4);
    ctx->d_fflags.reserve(static_cast<size_t>(fb) * 4);
    ctx->d_cand.reserve(slots * 4);
    ctx->d_npix.reserve(slots * 4);
    ctx->d_csidx.reserve((slots + 1) * 4);
    ctx->d_poff.reserve((slots + 1) * 4);
    ctx->d_slot_of.reserve(slots * 4);
    ctx->d_bpstat.reserve(BS_COUNT * 4);
    DevBuf *sl[] = {&ctx->d_slot_frame, &ctx->d_slot_id, &ctx->d_slot_np, &ctx->d_slot_pix, &ctx->d_slot_nv,
                    &ctx->d_slot_m,     &ctx->d_slot_ns, &ctx->d_slot_nn, &ctx->d_slot_toff, &ctx->d_slot_cov,
                    &ctx->d_kflag,      &ctx->d_ksize};
    for (DevBuf *b : sl) b->reserve(slots * 4);
    ctx->d_midx.reserve((slots + 1) * 4);
    ctx->d_moff.reserve((slots + 1) * 4);
    ctx->d_slot_box.reserve(slots * 6 * 4);
    ctx->d_cls_list.reserve((mc::kBpClasses + 1) * slots * 4);
    ctx->d_vox_order.reserve(slots * 4);
    ctx->d_vx_fb.reserve(2 * slots * 4);  // the two tiers' overflow lists
    ctx->d_scanm.reserve(4 * (slots / mc::kScanTile + 3) * 4);
    ctx->d_slot_grid.reserve(8 * slots * 8);
    // per-workgroup eps-neighbour lists, one region per size class (the classes run concurrently)
    ctx->d_nbl.reserve(nbl_offset(ctx, mc::kBpClasses) * 2);
    ctx->d_lean.reserve(lean_offset(ctx, mc::kBpClasses) * 4);
    if (ctx->bp_px_cap < px) {
        ctx->d_pix_list.reserve(px * 4);
        ctx->d_hkey.reserve(2 * px * 8);
        ctx->d_hvid.reserve(2 * px * 4);
        ctx->d_hfirst.reserve(2 * px * 4);
        fill_u32(s, ctx->d_hkey.ptr, 4 * px, 0xFFFFFFFFu);  // empty key, kept empty by k_bp_voxel
        fill_u32(s, ctx->d_hvid.ptr, 2 * px, 0xFFFFFFFFu);  // -1
        fill_u32(s, ctx->d_hfirst.ptr, 2 * px, 0x7FFFFFFFu);  // INT_MAX
        ctx->d_acc.reserve(px * 4 * 8);
        ctx->d_vx_pvid.reserve(px * 4);
        ctx->d_vx_list.reserve(px * 4);
        ctx->d_vox_entry.reserve(px * 4);
        ctx->d_vpts.reserve(px * 3 * 8);
        ctx->d_pcell.reserve(px * 8);
        ctx->d_pbkt.reserve(px * 4);
        ctx->d_bcnt.reserve(2 * px * 4);
        fill_u32(s, ctx->d_bcnt.ptr, 2 * px, 0u);  // kept zero by k_bp_denoise
        ctx->d_bstart.reserve((2 * px + slots + 1) * 4);
        ctx->d_blist.reserve(px * 4);
        ctx->d_ncnt.reserve(px * 4);
        ctx->d_par.reserve(px * 4);
        ctx->d_droot.reserve(px * 4);
        ctx->d_rnk.reserve(px * 4);
        ctx->d_lab.reserve(px * 4);
        ctx->d_ccnt.reserve((px + slots + 1) * 4);
        ctx->d_ssidx.reserve(px * 4);
        ctx->d_avg.reserve(px * 8);
        ctx->d_qpts.reserve(px * 3 * 4);
        ctx->bp_px_cap = px;
    }
    ctx->bp_f_cap = std::max(ctx->bp_f_cap, fb);
}

void bp_build_grid(mc_ctx *ctx, float radius, hipStream_t s)
{
    const int P = static_cast<int>(ctx->P_scene);
    const float inv = 1.0f / (2.0f * radius);
    const unsigned nb = static_cast<unsigned>(std::max(2 * P, 16));
    ctx->gnb = nb;
    const bool fresh = ctx->d_gcnt.bytes < (nb + 1) * 4ull;
    ctx->d_gcnt.reserve((nb + 1) * 4ull);
    if (fresh) MC_HIP(hipMemsetAsync(ctx->d_gcnt.ptr, 0, ctx->d_gcnt.bytes, s));  // kept zero by k_grid_scatter
    ctx->d_gstart.reserve((nb + 2) * 4ull);
    ctx->d_gbkt.reserve((P + 1) * 4ull);
    ctx->d_gcellk.reserve((P + 1) * 8ull);
    ctx->d_gpts.reserve((P + 1) * 16ull);
    ctx->d_gidx.reserve((P + 1) * 4ull);
    ctx->d_gcell.reserve((P + 1) * 8ull);
    ctx->d_gscan_tmp.reserve((2 * (nb / mc::kScanTile + 4) + 16) * 4ull);
    if (P) {
        hipLaunchKernelGGL(mc::k_grid_count, grid_for(P), dim3(256), 0, s, ctx->d_scene.as<float>(), P, inv, nb,
                           ctx->d_gcnt.as<int>(), ctx->d_gbkt.as<unsigned>(), ctx->d_gcellk.as<unsigned long long>());
    }
    mc::scan_large(s, ctx->d_gcnt.as<int>(), ctx->d_gstart.as<int>(), static_cast<int>(nb), ctx->d_gscan_tmp.as<int>());
    if (P)
        hipLaunchKernelGGL(mc::k_grid_scatter, grid_for(P), dim3(256), 0, s, ctx->d_scene.as<float>(), P,
                           ctx->d_gbkt.as<unsigned>(), ctx->d_gcellk.as<unsigned long long>(), ctx->d_gstart.as<int>(),
                           ctx->d_gcnt.as<int>(), ctx->d_gpts.as<float4>(), ctx->d_gidx.as<int>(),
                           ctx->d_gcell.as<unsigned long long>());
    ctx->grid_radius = radius;
}


// one LDS size class of the denoise: as many workgroups as are resident at once, each taking the
// class's slots from a ticket counter
// The k-NN ring search (k_bp_knn_ring) and the statistics / survivors (k_bp_denoise_tail) of every LDS
// class, once after the classes join, over one queue (queued per class behind each class kernel they
// measured 2 % slower at C3: the concurrent ring searches competed with the remaining classes,
// profiles/r04/r4e_tail_ab.jsonl)
void bp_denoise_tail_launch(mc_ctx *ctx, hipStream_t s, int ncap, int *st, const mc::BpDev &dv)
{
    auto ring = [&](auto kern, int wg_per_cu) {
        hipLaunchKernelGGL(kern, dim3(ctx->num_cu * wg_per_cu), dim3(256), 0, s, st + BS_DQ,
                           ctx->d_vx_pvid.as<int>(), ctx->d_slot_pix.as<int>(), ctx->d_slot_m.as<int>(), dv,
                           ctx->d_acc.as<double4>(), ctx->d_bstart.as<int>(), ctx->d_vx_list.as<int>(),
                           ctx->d_slot_grid.as<double>(), ctx->d_avg.as<double>(), st + BS_DNERR);
    };
    ring(mc::k_bp_knn_ring<4>, 8);  // (four waves per SIMD; at five or six, spilling: no faster)
    // a wave per slot whose ordered sums wait on latency: as many waves as its 45 VGPRs allow
    const int tail_wg = getenv("MC_BP_TAILWG") ? atoi(getenv("MC_BP_TAILWG")) : 8;
    hipLaunchKernelGGL(mc::k_bp_denoise_tail, dim3(ctx->num_cu * tail_wg), dim3(256), 0, s,
                       st + BS_CLS, ctx->d_cls_list.as<int>(), ncap, 0, mc::kBpClasses, ctx->d_slot_pix.as<int>(),
                       ctx->d_slot_m.as<int>(), dv, ctx->d_vpts.as<double>(), ctx->d_avg.as<double>(),
                       ctx->d_ssidx.as<int>(), ctx->d_qpts.as<float>(), ctx->d_slot_ns.as<int>(),
                       ctx->d_slot_box.as<float>());
}

template <int N>
void bp_denoise_class(mc_ctx *ctx, hipStream_t s, int cls, int ncap, int *st, const mc::BpDev &dv)
{
    using C = mc::BpLdsClass<N>;
    // the classes run concurrently: each has its own region of per-workgroup neighbour lists
    hipLaunchKernelGGL(mc::k_bp_denoise_lds<N>, dim3(ctx->num_cu * C::kWgPerCu * kBpOversub), dim3(C::T), 0, s, st + BS_CLS + cls,
                       ctx->d_cls_list.as<int>() + static_cast<size_t>(cls) * ncap, st + BS_TK + cls,
                       ctx->d_slot_pix.as<int>(), ctx->d_slot_nv.as<int>(), dv, ctx->d_vpts.as<double>(),
                       ctx->d_nbl.as<unsigned short>() + nbl_offset(ctx, cls), ctx->d_lean.as<int>() + lean_offset(ctx, cls),
                       ctx->d_slot_m.as<int>(), ctx->d_avg.as<double>(), ctx->d_ssidx.as<int>(),
                       ctx->d_acc.as<double4>(), ctx->d_bstart.as<int>(), ctx->d_vx_list.as<int>(),
                       ctx->d_vx_pvid.as<int>(), st + BS_DQ, static_cast<int>(std::min<size_t>(ctx->bp_px_cap, INT_MAX)),
                       ctx->d_slot_grid.as<double>(), st + BS_DNERR);
}
// MC_BP_DEBUG_SYNC=1: synchronise and report after every S1 group (diagnostics of a stalled batch)
void bp_debug_sync(hipStream_t s, const char *what)
{
    static const bool on = getenv("MC_BP_DEBUG_SYNC") != nullptr;
    if (!on) return;
    fprintf(stderr, "[mc bp] %s issued\n", what);
    MC_HIP(hipStreamSynchronize(s));
    MC_HIP(hipDeviceSynchronize());
    fprintf(stderr, "[mc bp] %s done\n", what);
}

}  // namespace

extern "C" {

void mc_bp_params_default(mc_bp_params *p)
{
    if (!p) return;
    p->depth_trunc = 20.0;
    p->voxel_size = 0.01;
    p->dbscan_eps = 0.04;
    p->component_min_fraction = 0.2;
    p->sor_std_ratio = 2.0;
    p->ball_radius = 0.01;
    p->coverage_threshold = 0.3;
    p->dbscan_min_points = 4;
    p->sor_neighbors = 20;
    p->ball_k = 20;
    p->few_points = 25;
}

int mc_scene_set_points(mc_ctx *ctx, int64_t num_points, const float *xyz, int on_device)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(num_points >= 0 && num_points < (int64_t(1) << 31) - 1, MC_ERR_UNSUPPORTED, "num_points out of range");
        MC_REQUIRE(num_points == 0 || xyz, MC_ERR_INVALID, "null points");
        hipStream_t s = ctx->stream;
        ctx->P_scene = num_points;
        ctx->d_scene.reserve((num_points + 1) * 12);
        if (num_points)
            MC_HIP(hipMemcpyAsync(ctx->d_scene.ptr, xyz, num_points * 12,
                                  on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
        ctx->have_points = true;
        ctx->have_bp = false;
        ctx->grid_radius = -1.f;  // the grid is built by the next mc_backproject
        MC_HIP(hipStreamSynchronize(s));
    });
}

// Per-frame host arrays -> one device array [F, frame_bytes]: the frames are copied by host
// threads into a pinned chunk while the previous chunk's DMA runs (pageable hipMemcpy would stage
// through the runtime's own buffers on one thread, and np.stack would add a full host copy).
// host frames of one mc_backproject_frames call; frames [0, staged) are on the device (or queued
// on ctx->copy before ctx->ev_up)
struct BpUpload {
    const void *const *depth;
    const void *const *seg;
    int staged;
    double raw_scale;  // > 0: depth frames are the PNGs' uint16 values, decoded on the copy stream
};

// frames [f_lo, f_hi) (frames[f] = host pointer of frame f) -> dst + f * frame_bytes, through the
// pinned ping-pong chunks: host threads fill one chunk while the DMA of the other runs on stream s
static void stage_frames(mc_ctx *ctx, const void *const *frames, size_t frame_bytes, int f_lo, int f_hi, char *dst,
                         hipStream_t s)
{
    if (f_hi <= f_lo || !frame_bytes) return;
    const size_t want = std::max<size_t>(frame_bytes, static_cast<size_t>(32) << 20);
    if (ctx->stage_bytes < want) {
        for (int b = 0; b < 2; b++) {
            if (ctx->stage_used[b]) MC_HIP(hipEventSynchronize(ctx->ev_stage[b]));
            if (ctx->h_stage[b]) MC_HIP(hipHostFree(ctx->h_stage[b]));
            ctx->h_stage[b] = nullptr;
            ctx->stage_used[b] = false;
        }
        ctx->stage_bytes = 0;
        for (int b = 0; b < 2; b++) {
            MC_HIP(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_stage[b]), want, hipHostMallocDefault));
            if (!ctx->ev_stage[b]) MC_HIP(hipEventCreateWithFlags(&ctx->ev_stage[b], hipEventDisableTiming));
        }
        ctx->stage_bytes = want;
    }
    int nthreads = static_cast<int>(std::min(8u, std::max(1u, std::thread::hardware_concurrency())));
    if (const char *e = getenv("MC_STAGE_THREADS")) nthreads = std::max(1, std::min(64, atoi(e)));
    const int per = static_cast<int>(std::max<size_t>(1, ctx->stage_bytes / frame_bytes));
    int b = 0;
    for (int f0 = f_lo; f0 < f_hi; f0 += per, b ^= 1) {
        const int n = std::min(per, f_hi - f0);
        if (ctx->stage_used[b]) MC_HIP(hipEventSynchronize(ctx->ev_stage[b]));  // its last DMA is done
        char *buf = ctx->h_stage[b];
        const size_t total = static_cast<size_t>(n) * frame_bytes;
        auto copy_range = [&](size_t lo, size_t hi) {
            while (lo < hi) {
                const size_t f = lo / frame_bytes, o = lo % frame_bytes;
                const size_t len = std::min(hi - lo, frame_bytes - o);
                memcpy(buf + lo, static_cast<const char *>(frames[f0 + f]) + o, len);
                lo += len;
            }
        };
        const int nt = static_cast<int>(std::min<size_t>(nthreads, std::max<size_t>(1, total >> 22)));  // >= 4 MB each
        if (nt <= 1) {
            copy_range(0, total);
        } else {
            std::vector<std::thread> th;
            const size_t step = (total + nt - 1) / nt;
            for (int t = 1; t < nt; t++) th.emplace_back(copy_range, std::min(total, t * step), std::min(total, (t + 1) * step));
            copy_range(0, std::min(total, step));
            for (auto &x : th) x.join();
        }
        MC_HIP(hipMemcpyAsync(dst + static_cast<size_t>(f0) * frame_bytes, buf, total, hipMemcpyHostToDevice, s));
        MC_HIP(hipEventRecord(ctx->ev_stage[b], s));
        ctx->stage_used[b] = true;
    }
}

static int backproject_frames_impl(mc_ctx *ctx, int32_t num_frames, int32_t height, int32_t width,
                                   const void *const *depth_frames, double raw_scale, const uint8_t *const *seg_frames,
                                   const double *intrinsics, const double *poses, const mc_bp_params *params)
{
    const int rc = guarded(ctx, [&] {
        MC_REQUIRE(raw_scale >= 0.0 && std::isfinite(raw_scale), MC_ERR_INVALID, "bad depth_scale");
        MC_REQUIRE(num_frames >= 0 && height > 0 && width > 0, MC_ERR_INVALID, "bad frame sizes");
        MC_REQUIRE(num_frames == 0 || (depth_frames && seg_frames && intrinsics && poses), MC_ERR_INVALID,
                   "null frame arrays");
        for (int f = 0; f < num_frames; f++)
            MC_REQUIRE(depth_frames[f] && seg_frames[f], MC_ERR_INVALID, "null frame array");
        const int F = num_frames;
        const size_t HW = static_cast<size_t>(height) * width;
        if (!F) return;
        hipStream_t s = ctx->stream;
        ctx->d_in_depth.reserve(F * HW * 4);
        ctx->d_in_seg.reserve(F * HW);
        if (raw_scale > 0.0) ctx->d_in_raw.reserve(F * HW * 2);
        ctx->d_in_intr.reserve(F * 4 * 8ull);
        ctx->d_in_pose.reserve(F * 16 * 8ull);
        MC_HIP(hipMemcpyAsync(ctx->d_in_intr.ptr, intrinsics, F * 4 * 8ull, hipMemcpyHostToDevice, s));
        MC_HIP(hipMemcpyAsync(ctx->d_in_pose.ptr, poses, F * 16 * 8ull, hipMemcpyHostToDevice, s));
        if (!ctx->copy) {
            MC_HIP(hipStreamCreateWithFlags(&ctx->copy, hipStreamNonBlocking));
            MC_HIP(hipEventCreateWithFlags(&ctx->ev_up, hipEventDisableTiming));
        }
    });
    if (rc != MC_OK) return rc;
    if (!num_frames) {
        static const float zf = 0.f;
        static const uint8_t zs = 0;
        static const double zd[16] = {};
        return mc_backproject(ctx, 0, height, width, &zf, &zs, zd, zd, 0, params);
    }
    // the frames are staged by the S1 batch loop itself: batch b + 1's while batch b computes
    BpUpload up{depth_frames, reinterpret_cast<const void *const *>(seg_frames), 0, raw_scale};
    ctx->bp_up = &up;
    const int rc2 = mc_backproject(ctx, num_frames, height, width, ctx->d_in_depth.as<float>(),
                                   ctx->d_in_seg.as<uint8_t>(), ctx->d_in_intr.as<double>(),
                                   ctx->d_in_pose.as<double>(), 1, params);
    ctx->bp_up = nullptr;
    (void)hipStreamSynchronize(ctx->copy);  // no DMA into d_in_* outlives the call (error paths)
    return rc2;
}

int mc_backproject_frames(mc_ctx *ctx, int32_t num_frames, int32_t height, int32_t width,
                          const float *const *depth_frames, const uint8_t *const *seg_frames,
                          const double *intrinsics, const double *poses, const mc_bp_params *params)
{
    return backproject_frames_impl(ctx, num_frames, height, width, reinterpret_cast<const void *const *>(depth_frames),
                                   0.0, seg_frames, intrinsics, poses, params);
}

int mc_backproject_frames_raw(mc_ctx *ctx, int32_t num_frames, int32_t height, int32_t width,
                              const uint16_t *const *depth_frames, double depth_scale,
                              const uint8_t *const *seg_frames, const double *intrinsics, const double *poses,
                              const mc_bp_params *params)
{
    if (!(depth_scale > 0.0)) return guarded(ctx, [&] { MC_REQUIRE(false, MC_ERR_INVALID, "depth_scale must be > 0"); });
    return backproject_frames_impl(ctx, num_frames, height, width, reinterpret_cast<const void *const *>(depth_frames),
                                   depth_scale, seg_frames, intrinsics, poses, params);
}

int mc_backproject(mc_ctx *ctx, int32_t num_frames, int32_t height, int32_t width, const float *depth,
                   const uint8_t *seg, const double *intrinsics, const double *poses, int on_device,
                   const mc_bp_params *params)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_points, MC_ERR_STATE, "mc_backproject before mc_scene_set_points");
        MC_REQUIRE(num_frames >= 0 && height > 0 && width > 0, MC_ERR_INVALID, "bad frame sizes");
        MC_REQUIRE(num_frames == 0 || (depth && seg && intrinsics && poses), MC_ERR_INVALID, "null frame arrays");
        MC_REQUIRE(static_cast<int64_t>(height) * width < (int64_t(1) << 31), MC_ERR_UNSUPPORTED, "image too large");
        mc_bp_params prm;
        if (params) prm = *params;
        else mc_bp_params_default(&prm);
        MC_REQUIRE(prm.sor_neighbors >= 1 && prm.sor_neighbors <= mc::kBpKnnMax, MC_ERR_UNSUPPORTED,
                   "sor_neighbors must be in [1, 20]");
        MC_REQUIRE(prm.ball_k >= 1 && prm.ball_k <= mc::kBpBallMax, MC_ERR_UNSUPPORTED, "ball_k must be in [1, 32]");
        MC_REQUIRE(prm.voxel_size > 0 && prm.dbscan_eps > 0 && prm.ball_radius > 0, MC_ERR_INVALID, "bad radii");
        hipStream_t s = ctx->stream;
        const int F = num_frames, H = height, W = width;
        const size_t HW = static_cast<size_t>(H) * W;
        const int nbands = (H + mc::kBpBand - 1) / mc::kBpBand;
        ctx->have_bp = false;
        ctx->bp_F = F;
        ctx->bp_err_frame = -1;
        ctx->bp_col.clear();
        ctx->bp_label.clear();
        ctx->bp_off.assign(1, 0);
        ctx->bp_stats.clear();
        ctx->bp_nnz = 0;
        const float rf = static_cast<float>(prm.ball_radius);
        if (ctx->grid_radius != rf) {  // a new scene (mc_scene_set_points) or radius: the 2r scene grid
            TimedScope ts(ctx->timer, s, "bp_grid");
            bp_build_grid(ctx, rf, s);
        }

        const float *dep = depth;
        const uint8_t *sg = seg;
        const double *Kp = intrinsics, *Tp = poses;
        if (!on_device && F) {
            ctx->d_in_depth.reserve(F * HW * 4);
            ctx->d_in_seg.reserve(F * HW);
            ctx->d_in_intr.reserve(F * 4 * 8ull);
            ctx->d_in_pose.reserve(F * 16 * 8ull);
            MC_HIP(hipMemcpyAsync(ctx->d_in_depth.ptr, depth, F * HW * 4, hipMemcpyHostToDevice, s));
            MC_HIP(hipMemcpyAsync(ctx->d_in_seg.ptr, seg, F * HW, hipMemcpyHostToDevice, s));
            MC_HIP(hipMemcpyAsync(ctx->d_in_intr.ptr, intrinsics, F * 4 * 8ull, hipMemcpyHostToDevice, s));
            MC_HIP(hipMemcpyAsync(ctx->d_in_pose.ptr, poses, F * 16 * 8ull, hipMemcpyHostToDevice, s));
            dep = ctx->d_in_depth.as<float>();
            sg = ctx->d_in_seg.as<uint8_t>();
            Kp = ctx->d_in_intr.as<double>();
            Tp = ctx->d_in_pose.as<double>();
        }
        // test knob: smallest denoise size class (0 = by size; 3 = the lean LDS class, 4 = the
        // global-memory kernel for every slot)
        int min_cls = 0;
        if (const char *e = getenv("MC_BP_MIN_CLASS")) min_cls = std::min(mc::kBpClasses, std::max(0, atoi(e)));
        // test knob: MC_VX_GLOBAL=1 hands every slot to the global-hash voxel kernel, =2 to the second
        // LDS tier
        const int vx_global = getenv("MC_VX_GLOBAL") ? atoi(getenv("MC_VX_GLOBAL")) : 0;
        // frames per batch: bounded pixel capacity of the per-slot arrays (≈ 200 B of per-batch arrays
        // per pixel).  Large batches amortise every group's slot tail and the per-batch sync (C3 E2E:
        // 192 M pixels 215 ms, 400 M 184 ms, 600 M 175 ms per scene in round 2; 1 G 115 ms against
        // 118 ms at the old 640 M / 45 % cap in round 3, profiles/r03/ab19_batch_pixels.jsonl), so the
        // batch takes up to 1 G pixels or 65 % of the free HBM (≈ 170 GB of a fresh 288 GB device),
        // whichever is less; the frames are then dealt into equal batches, so that no batch is a small
        // remainder with its own tails
        // The per-batch arrays take at most the context's HBM budget (mc_ctx_set_memory_budget), by
        // default 40 % of the device or 65 % of what is free (plus what this context already holds),
        // whichever is less, so a caller's own allocator keeps room (a fresh 288 GB MI355X: ~115 GB,
        // ~530 M pixels per batch); a caller that owns the device (bench.py) sets a larger one.
        // frame pixels per batch: below 2^31 (int positions), and within the byte budget at the
        // expected mask-pixel share (C3: 0.23 of the frame pixels, so two batches instead of six; the
        // per-batch tails and syncs cost ~3 ms each, profiles/r05/r5s_*)
        size_t budget = (static_cast<size_t>(1) << 31) - 1;
        // test knob: MC_BP_MASK_FRAC sets the expected share (a small one forces the grow-and-redo path)
        if (const char *e = getenv("MC_BP_MASK_FRAC")) ctx->bp_mfrac = atof(e);
        const double mfrac = std::min(1.0, std::max(ctx->bp_mfrac, 1e-4));
        size_t bud_bytes = 0;  // the per-batch arrays' byte budget (also bounds the grow-and-redo below)
        {
            const size_t held = ctx->bp_px_cap * kBpBytesPerMaskPixel + ctx->bp_fpx_cap * kBpBytesPerFramePixel;
            size_t bytes = static_cast<size_t>(ctx->mem_budget);
            if (ctx->mem_budget <= 0) {
                size_t free_b = 0, total_b = 0;
                bytes = held;
                if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && total_b)
                    bytes = std::min(total_b / 100 * 40, (free_b + held) / 100 * 65);
            }
            bud_bytes = bytes;
            const double per_px = static_cast<double>(kBpBytesPerFramePixel) + mfrac * kBpBytesPerMaskPixel;
            budget = std::max<size_t>(HW, std::min(budget, static_cast<size_t>(static_cast<double>(bytes) / per_px)));
        }
        const bool fixed_batch = getenv("MC_BP_BATCH_PIXELS") != nullptr;
        if (const char *e = getenv("MC_BP_BATCH_PIXELS")) budget = std::max<size_t>(1, strtoull(e, nullptr, 10));
        BpUpload *const up = on_device ? ctx->bp_up : nullptr;
        int FB = static_cast<int>(std::max<size_t>(1, std::min<size_t>(std::max(F, 1), budget / HW)));
        {
            const int nb = (std::max(F, 1) + FB - 1) / FB;
            FB = (std::max(F, 1) + nb - 1) / nb;
        }
        // frames arriving from the host: batch b + 1's upload runs under batch b's compute.  Splitting a
        // scene that fits one batch into more batches only to overlap its upload did not pay (C2 API
        // path: 1 batch 44.9 ms, 8 batches 46.2 ms, profiles/r03/api/), so by default only scenes of
        // several batches overlap (C3: 7); MC_BP_UPLOAD_BATCHES=n forces at least n batches
        if (up) {
            int nb = 1;
            if (const char *e = getenv("MC_BP_UPLOAD_BATCHES")) nb = std::max(1, atoi(e));
            FB = std::max(1, std::min(FB, (F + nb - 1) / nb));
        }
        // stage the host frames [up->staged, f_hi) on the copy stream
        auto upload_to = [&](int f_hi) {
            if (!up || f_hi <= up->staged) return;
            if (up->raw_scale > 0.0) {  // 2-byte frames, then float32(u16 / scale) on the copy stream
                stage_frames(ctx, up->depth, HW * 2, up->staged, f_hi, static_cast<char *>(ctx->d_in_raw.ptr), ctx->copy);
                const int64_t total = static_cast<int64_t>(f_hi - up->staged) * static_cast<int64_t>(HW);
                hipLaunchKernelGGL(mc::k_frames_decode, grid_for(total, 256, 16384), dim3(256), 0, ctx->copy, total, H, W,
                                   1, 1, ctx->d_in_raw.as<unsigned short>() + static_cast<size_t>(up->staged) * HW,
                                   up->raw_scale, static_cast<const unsigned char *>(nullptr),
                                   static_cast<const int *>(nullptr), static_cast<const int *>(nullptr),
                                   ctx->d_in_depth.as<float>() + static_cast<size_t>(up->staged) * HW,
                                   static_cast<unsigned char *>(nullptr));
                MC_HIP(hipGetLastError());
            } else {
                stage_frames(ctx, up->depth, HW * 4, up->staged, f_hi, static_cast<char *>(ctx->d_in_depth.ptr), ctx->copy);
            }
            stage_frames(ctx, up->seg, HW, up->staged, f_hi, static_cast<char *>(ctx->d_in_seg.ptr), ctx->copy);
            MC_HIP(hipEventRecord(ctx->ev_up, ctx->copy));
            up->staged = f_hi;
        };
        // mask-pixel capacity for a batch of FB frames at the expected share (+ 1/16 and a frame's worth)
        auto mask_cap = [&](double frac) {
            const double fpx = static_cast<double>(FB) * static_cast<double>(HW);
            return static_cast<size_t>(std::min(fpx, frac * fpx * 1.0625 + static_cast<double>(HW))) + 1024;
        };
        bp_reserve(ctx, FB, H, W, nbands, mask_cap(mfrac), s);
        double mfrac_seen = 0.0;
        const int PW = static_cast<int>((ctx->P_scene + 63) / 64) + 1;
        const int qgrid = ctx->num_cu * 6;  // one bitmap per query workgroup (its largest grid)
        if (ctx->d_bpbm.bytes < static_cast<size_t>(qgrid) * PW * 8) {
            ctx->d_bpbm.reserve(static_cast<size_t>(qgrid) * PW * 8);
            MC_HIP(hipMemsetAsync(ctx->d_bpbm.ptr, 0, ctx->d_bpbm.bytes, s));  // kept zero by k_bp_query
            ctx->bp_bm_blocks = qgrid;
        }
        size_t tmp_cap = std::max<size_t>(ctx->d_tmp.bytes / 4, std::max<size_t>(1 << 20, ctx->bp_px_cap));
        ctx->d_tmp.reserve(tmp_cap * 4);

        mc::BpDev dv;
        dv.trunc = prm.depth_trunc;
        dv.vs = prm.voxel_size;
        dv.rvs = 1.0 / prm.voxel_size;  // (IEEE division on the host: RN(1 / vs), div_rn's reciprocal)
        dv.eps2 = prm.dbscan_eps * prm.dbscan_eps;
        // k-NN pre-selection radii (fractions of eps, ascending, < 1): any choice gives the same
        // results (the smallest radius holding >= k kept points is used); MC_KNN_RADII="a,b,c" tunes
        double kfr[3] = {0.6, 0.75, 0.9};
        if (const char *e = getenv("MC_KNN_RADII")) {
            double a[3];
            if (sscanf(e, "%lf,%lf,%lf", &a[0], &a[1], &a[2]) == 3 && 0 < a[0] && a[0] < a[1] && a[1] < a[2] && a[2] < 1)
                for (int i = 0; i < 3; i++) kfr[i] = a[i];
        }
        for (int i = 0; i < 3; i++) dv.knn_r2[i] = (kfr[i] * prm.dbscan_eps) * (kfr[i] * prm.dbscan_eps);
        dv.ce = prm.dbscan_eps * 1.01;
        dv.frac = prm.component_min_fraction;
        dv.std_ratio = prm.sor_std_ratio;
        dv.cov = prm.coverage_threshold;
        dv.r2 = rf * rf;
        dv.scene_inv = 1.0f / (2.0f * rf);
        dv.minpts = prm.dbscan_min_points;
        dv.knn = prm.sor_neighbors;
        dv.kball = prm.ball_k;
        dv.few = prm.few_points;
        dv.H = H;
        dv.W = W;
        dv.nbands = nbands;
        // the pixel kernels' uchar4 / float4 loads need aligned frames (a caller's tensor view may start
        // at any element); every batch starts HW pixels further on, a multiple of 4 when W is
        // test knob: eps lists read only up to MC_BP_NBCAP entries (the rest take the cell walks)
        dv.nbcap = mc::kBpNbCap;
        if (const char *e = getenv("MC_BP_NBCAP")) dv.nbcap = std::min(mc::kBpNbCap, std::max(1, atoi(e)));
        dv.vec4 = (W % 4 == 0 && reinterpret_cast<uintptr_t>(dep) % 16 == 0 && reinterpret_cast<uintptr_t>(sg) % 4 == 0)
                      ? 1 : 0;

        int *st = ctx->d_bpstat.as<int>();
        if (!ctx->h_bpstat) MC_HIP(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_bpstat), BS_COUNT * sizeof(int),
                                                 hipHostMallocDefault));
        int *const hs = ctx->h_bpstat;  // pinned
        if (!ctx->ev_pack) MC_HIP(hipEventCreateWithFlags(&ctx->ev_pack, hipEventDisableTiming));
        // the host side of a batch (its masks and statistics appended from h_bppack) runs while the
        // next batch computes: the batch's copy into h_bppack is stream-ordered before the next batch,
        // whose own copy comes only after its statistics sync, i.e. after this unpack
        struct PendingBatch {
            bool valid = false;
            int b0 = 0, Mb = 0, NS = 0, nnzb = 0;
            int64_t nnz_base = 0;
        } pend;
        auto unpack = [&]() {
            if (!pend.valid) return;
            MC_HIP(hipEventSynchronize(ctx->ev_pack));
            const int Mb = pend.Mb, NS = pend.NS, nnzb = pend.nnzb, bb = pend.b0;
            const int *col = ctx->h_bppack, *lab = col + Mb, *off = lab + Mb;
            const int *sf = off + Mb, *sid = sf + NS, *snp = sid + NS, *snv = snp + NS, *sm = snv + NS,
                      *sns = sm + NS, *scov = sns + NS, *snn = scov + NS;
            for (int g = 0; g < Mb; g++) {
                ctx->bp_col.push_back(bb + col[g]);
                ctx->bp_label.push_back(lab[g]);
            }
            for (int g = 0; g < Mb; g++) ctx->bp_off.push_back(pend.nnz_base + (g + 1 < Mb ? off[g + 1] : nnzb));
            for (int x = 0; x < NS; x++) {
                const int kept = snn[x] >= 0;
                const int row[MC_BP_NSTAT] = {bb + sf[x], sid[x], snp[x], snv[x], sm[x], sns[x], -1,
                                              sns[x] >= prm.few_points ? scov[x] : 0, kept ? snn[x] : 0, kept};
                ctx->bp_stats.insert(ctx->bp_stats.end(), row, row + MC_BP_NSTAT);
            }
            pend.valid = false;
        };
        for (int b0 = 0; b0 < F;) {
            const int fb = std::min(FB, F - b0);
            if (up) {
                upload_to(b0 + fb);
                MC_HIP(hipStreamWaitEvent(s, ctx->ev_up, 0));
            }
            const float *dB = dep + b0 * HW;
            const uint8_t *sB = sg + b0 * HW;
            const double *KB = Kp + 4 * static_cast<size_t>(b0), *TB = Tp + 16 * static_cast<size_t>(b0);
            const int nslot = fb * 256;
            {
                TimedScope ts(ctx->timer, s, "bp_pixels");
                hipLaunchKernelGGL(mc::k_bp_stat_init, dim3(1), dim3(64), 0, s, st, static_cast<int>(BS_COUNT));
                MC_HIP(hipMemsetAsync(ctx->d_present.ptr, 0, fb * 8 * 4, s));
                MC_HIP(hipMemsetAsync(ctx->d_fflags.ptr, 0, fb * 4, s));
                hipLaunchKernelGGL(mc::k_bp_count, dim3(nbands, fb), dim3(256), 0, s, dB, sB, TB, dv,
                                   ctx->d_band.as<int>(), ctx->d_present.as<unsigned>(), ctx->d_fflags.as<int>(),
                                   ctx->d_bpvid.as<unsigned char>());
                hipLaunchKernelGGL(mc::k_bp_frames, dim3(fb), dim3(1024), 0, s, ctx->d_band.as<int>(),
                                   ctx->d_present.as<unsigned>(), ctx->d_fflags.as<int>(), dv, ctx->d_cand.as<int>(),
                                   ctx->d_npix.as<int>(), st + BS_ERRF);
                mc::scan_device_multi(s, nullptr, nslot, ctx->d_scanm.as<int>(), ctx->d_cand.as<int>(),
                                      ctx->d_csidx.as<int>(), st + BS_NS, ctx->d_npix.as<int>(), ctx->d_poff.as<int>(),
                                      st + BS_NPX);
                hipLaunchKernelGGL(mc::k_bp_slots, grid_for(nslot), dim3(256), 0, s, ctx->d_cand.as<int>(),
                                   ctx->d_csidx.as<int>(), ctx->d_npix.as<int>(), ctx->d_poff.as<int>(), nslot,
                                   ctx->d_slot_of.as<int>(), ctx->d_slot_frame.as<int>(), ctx->d_slot_id.as<int>(),
                                   ctx->d_slot_np.as<int>(), ctx->d_slot_pix.as<int>(), st + BS_NPX,
                                   static_cast<int>(std::min<size_t>(ctx->bp_px_cap, INT_MAX)), st + BS_NS, st + BS_PXOVF);
                hipLaunchKernelGGL(mc::k_bp_compact, dim3(nbands, fb), dim3(256), 0, s, ctx->d_bpvid.as<unsigned char>(),
                                   ctx->d_band.as<int>(),
                                   ctx->d_slot_of.as<int>(), ctx->d_slot_pix.as<int>(), dv,
                                   ctx->d_pix_list.as<unsigned>());
                bp_debug_sync(s, "bp_pixels");
            }
            {
                TimedScope ts(ctx->timer, s, "bp_voxel");
                hipLaunchKernelGGL(mc::k_bp_vox_order, dim3(1), dim3(1024), 0, s, st + BS_NS, ctx->d_slot_np.as<int>(),
                                   ctx->d_vox_order.as<int>());
                int *fb1 = ctx->d_vx_fb.as<int>(), *fb2 = fb1 + slots_cap(FB);
                auto tier1 = [&](auto kern, int wg_per_cu) {
                    hipLaunchKernelGGL(kern, dim3(ctx->num_cu * wg_per_cu), dim3(mc::kVxT), 0, s,
                                       st + BS_NS, ctx->d_vox_order.as<int>(), ctx->d_slot_frame.as<int>(),
                                       ctx->d_slot_np.as<int>(), ctx->d_slot_pix.as<int>(), ctx->d_pix_list.as<unsigned>(), dB,
                                       KB, TB, dv, ctx->d_vx_pvid.as<int>(), ctx->d_vpts.as<double>(),
                                       ctx->d_slot_nv.as<int>(), fb1, st + BS_VXFB, vx_global >= 1 ? 1 : 0,
                                       ctx->d_slot_grid.as<double>());
                };
                auto tier2 = [&](auto kern) {
                    hipLaunchKernelGGL(kern, dim3(ctx->num_cu), dim3(mc::kVxT2), 0, s,
                                       st + BS_VXFB, fb1, ctx->d_slot_frame.as<int>(), ctx->d_slot_np.as<int>(),
                                       ctx->d_slot_pix.as<int>(), ctx->d_pix_list.as<unsigned>(), dB, KB, TB, dv,
                                       ctx->d_vx_pvid.as<int>(), ctx->d_vpts.as<double>(), ctx->d_slot_nv.as<int>(), fb2,
                                       st + BS_VXFB2, vx_global == 1 ? 1 : 0, ctx->d_slot_grid.as<double>());
                };
                // five workgroups per CU (32 KB of LDS, <= 96 VGPRs each) for the first tier
                tier1(mc::k_bp_voxel_lds<mc::kVxT, mc::kVxH, mc::kVxV, 0, mc::kVxWpe>, mc::kVxWpe);
                tier2(mc::k_bp_voxel_lds<mc::kVxT2, mc::kVxH2, mc::kVxV2, mc::kVxL2>);
                hipLaunchKernelGGL(mc::k_bp_voxel, dim3(ctx->num_cu), dim3(256), 0, s, st + BS_VXFB2,
                                   fb2, ctx->d_slot_frame.as<int>(), ctx->d_slot_np.as<int>(),
                                   ctx->d_slot_pix.as<int>(), ctx->d_pix_list.as<unsigned>(), dB, KB, TB, dv,
                                   ctx->d_hkey.as<unsigned long long>(), ctx->d_hvid.as<int>(), ctx->d_hfirst.as<int>(),
                                   ctx->d_vox_entry.as<int>(), ctx->d_acc.as<double>(), ctx->d_vpts.as<double>(),
                                   ctx->d_slot_nv.as<int>(), st + BS_VOXERR, ctx->d_slot_grid.as<double>());
                bp_debug_sync(s, "bp_voxel");
            }
            {
                TimedScope ts(ctx->timer, s, "bp_denoise");
                const int ncap = static_cast<int>(slots_cap(fb));
                // largest first again, now by voxel count (the denoise's and the query's cost)
                hipLaunchKernelGGL(mc::k_bp_vox_order, dim3(1), dim3(1024), 0, s, st + BS_NS, ctx->d_slot_nv.as<int>(),
                                   ctx->d_vox_order.as<int>());
                hipLaunchKernelGGL(mc::k_bp_classify, dim3(64), dim3(256), 0, s, st + BS_NS, ctx->d_slot_nv.as<int>(),
                                   ctx->d_vox_order.as<int>(), ncap, min_cls, st + BS_CLS, ctx->d_cls_list.as<int>());
                // the few slots beyond the LDS classes run on the side stream, beside the classes
                MC_HIP(hipEventRecord(ctx->ev_fork, s));
                MC_HIP(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
                bp_denoise_class<16384>(ctx, ctx->side, 5, ncap, st, dv);  // few, large slots
                hipLaunchKernelGGL(mc::k_bp_denoise, dim3(ctx->num_cu), dim3(256), 0, ctx->side, st + BS_CLS + mc::kBpClasses,
                                   ctx->d_cls_list.as<int>() + mc::kBpClasses * static_cast<size_t>(ncap), ctx->d_slot_pix.as<int>(), ctx->d_slot_nv.as<int>(), dv, ctx->d_vpts.as<double>(),
                                   ctx->d_pcell.as<unsigned long long>(), ctx->d_pbkt.as<int>(), ctx->d_bcnt.as<int>(),
                                   ctx->d_bstart.as<int>(), ctx->d_blist.as<int>(), ctx->d_ncnt.as<int>(),
                                   ctx->d_par.as<int>(), ctx->d_droot.as<int>(), ctx->d_rnk.as<int>(),
                                   ctx->d_lab.as<int>(), ctx->d_ccnt.as<int>(), ctx->d_ssidx.as<int>(),
                                   ctx->d_avg.as<double>(), ctx->d_qpts.as<float>(), ctx->d_slot_m.as<int>(),
                                   ctx->d_slot_ns.as<int>(), ctx->d_slot_box.as<float>());
                MC_HIP(hipEventRecord(ctx->ev_join, ctx->side));
                // the LDS classes side by side, each on its own stream: a class with few slots
                // (the large ones) leaves most CUs to the others instead of serialising the batch
                for (int c = 0; c < mc::kBpStreamClasses; c++) MC_HIP(hipStreamWaitEvent(ctx->cls_stream[c], ctx->ev_fork, 0));
                bp_denoise_class<3072>(ctx, ctx->cls_stream[3], 3, ncap, st, dv);
                bp_denoise_class<4096>(ctx, ctx->cls_stream[4], 4, ncap, st, dv);
                bp_denoise_class<2048>(ctx, ctx->cls_stream[2], 2, ncap, st, dv);
                bp_denoise_class<1024>(ctx, ctx->cls_stream[1], 1, ncap, st, dv);
                bp_denoise_class<512>(ctx, ctx->cls_stream[0], 0, ncap, st, dv);
                for (int c = 0; c < mc::kBpStreamClasses; c++) {
                    MC_HIP(hipEventRecord(ctx->ev_cls[c], ctx->cls_stream[c]));
                    MC_HIP(hipStreamWaitEvent(s, ctx->ev_cls[c], 0));
                }
                MC_HIP(hipStreamWaitEvent(s, ctx->ev_join, 0));
                // the deferred points' ring search, then every LDS-class slot's statistics and survivors
                bp_denoise_tail_launch(ctx, s, ncap, st, dv);
                bp_debug_sync(s, "bp_denoise");
            }
            {
                TimedScope ts(ctx->timer, s, "bp_query");
                auto query = [&](auto kern, int grid) {
                hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, st + BS_NS,
                                   ctx->d_slot_pix.as<int>(), ctx->d_slot_ns.as<int>(), ctx->d_slot_box.as<float>(),
                                   ctx->d_qpts.as<float>(), dv, ctx->d_gpts.as<float4>(), ctx->d_gidx.as<int>(),
                                   ctx->d_gcell.as<unsigned long long>(), ctx->d_gstart.as<int>(), ctx->gnb,
                                   ctx->d_bpbm.as<unsigned long long>(), PW, ctx->d_tmp.as<int>(),
                                   static_cast<int>(std::min<size_t>(tmp_cap, INT_MAX)), st + BS_TOP,
                                   ctx->d_slot_nn.as<int>(), ctx->d_slot_toff.as<int>(), ctx->d_slot_cov.as<int>(),
                                   st + BS_OVF, ctx->d_vox_order.as<int>());
                };
                // the query waits on dependent cell-range and point loads: as many waves as the
                // registers allow (the 20-entry best list of ball_k <= 20: 76 VGPRs, six workgroups per
                // CU, C3 query 8.4 -> 6.5 ms per scene; 32 entries: 89 VGPRs, five)
                if (prm.ball_k <= 20) query(mc::k_bp_query<1, 20>, ctx->num_cu * 6);
                else query(mc::k_bp_query<1, mc::kBpBallMax>, ctx->num_cu * 5);
                bp_debug_sync(s, "k_bp_query");
                hipLaunchKernelGGL(mc::k_bp_keepflags, grid_for(nslot), dim3(256), 0, s, st + BS_NS,
                                   ctx->d_slot_nn.as<int>(), ctx->d_kflag.as<int>(), ctx->d_ksize.as<int>());
                mc::scan_device_multi(s, st + BS_NS, nslot, ctx->d_scanm.as<int>(), ctx->d_kflag.as<int>(),
                                      ctx->d_midx.as<int>(), st + BS_M, ctx->d_ksize.as<int>(), ctx->d_moff.as<int>(),
                                      st + BS_NNZ);
                bp_debug_sync(s, "bp_query");
            }
            MC_HIP(hipMemcpyAsync(hs, st, BS_COUNT * 4, hipMemcpyDeviceToHost, s));
            upload_to(std::min(F, b0 + fb + FB));  // the host copies the next batch while this one computes
            unpack();                               // and appends the previous batch's results
            MC_HIP(hipStreamSynchronize(s));
            ctx->timer.collect();
            if (hs[BS_ERRF] != INT_MAX) {
                ctx->bp_err_frame = b0 + hs[BS_ERRF];
                throw McError{MC_ERR_INVALID, "frame " + std::to_string(b0 + hs[BS_ERRF]) +
                                                  ": depth pixel equal to depth_trunc (the reference raises "
                                                  "IndexError at utils/mask_backprojection.py:100)"};
            }
            MC_REQUIRE(!(hs[BS_VOXERR] & 2), MC_ERR_HIP, "voxel hash table not empty at slot start (internal error)");
            MC_REQUIRE(hs[BS_DNERR] == 0, MC_ERR_HIP,
                       "denoise: k-NN ring-search queue " + std::string(hs[BS_DNERR] & 1 ? "entry" : "region") +
                           " out of range (internal error)");
            MC_REQUIRE(hs[BS_VOXERR] == 0, MC_ERR_UNSUPPORTED, "voxel index beyond 2^21 per axis");
            if (hs[BS_PXOVF]) {  // more mask pixels than the capacity (nothing past the pixel lists ran): grow, redo
                const double frac = static_cast<double>(hs[BS_NPX]) / (static_cast<double>(fb) * HW);
                ctx->bp_mfrac = std::max(ctx->bp_mfrac, frac);
                // within the byte budget: at the observed share the batch takes fewer frames (a denser
                // scene than the share learned so far), instead of arrays up to 1 / share times the budget
                const int fb_was = FB;
                if (!fixed_batch) {
                    const double per_px = static_cast<double>(kBpBytesPerFramePixel) +
                                          std::min(1.0, frac * 1.0625 + 1.0 / FB) * kBpBytesPerMaskPixel;
                    const double fit = std::floor(static_cast<double>(bud_bytes) / (per_px * static_cast<double>(HW)));
                    FB = std::max(1, std::min(FB, static_cast<int>(std::min(fit, 1e9))));
                }
                // the same frames again: room for every pixel they listed; fewer frames: the share's room
                // (another overflow shrinks the batch or grows the arrays again, so the redo terminates)
                bp_reserve(ctx, FB, H, W, nbands,
                           FB < fb_was ? mask_cap(frac) : std::max(mask_cap(frac), static_cast<size_t>(hs[BS_NPX]) + 1024), s);
                ctx->bp_redo++;
                continue;
            }
            mfrac_seen = std::max(mfrac_seen, static_cast<double>(hs[BS_NPX]) / (static_cast<double>(fb) * HW));
            if (hs[BS_OVF]) {  // neighbour sets overflowed tmp: grow and redo the batch
                tmp_cap = static_cast<size_t>(hs[BS_TOP]) + (static_cast<size_t>(hs[BS_TOP]) >> 1) + 1024;
                ctx->d_tmp.reserve(tmp_cap * 4);
                continue;
            }
            const int NS = hs[BS_NS], Mb = hs[BS_M], nnzb = hs[BS_NNZ];
            ctx->d_out_col.reserve((Mb + 1) * 4);
            ctx->d_out_label.reserve((Mb + 1) * 4);
            ctx->d_out_off.reserve((Mb + 1) * 4);
            grow_keep(ctx->d_bp_pts, (ctx->bp_nnz + nnzb + 1) * 4, ctx->bp_nnz * 4, s);
            {
                TimedScope ts(ctx->timer, s, "bp_query");
                hipLaunchKernelGGL(mc::k_bp_emit, grid_for(std::max(NS, 1), 4, 4096), dim3(256), 0, s, st + BS_NS,
                                   ctx->d_slot_frame.as<int>(), ctx->d_slot_id.as<int>(), ctx->d_slot_nn.as<int>(),
                                   ctx->d_slot_toff.as<int>(), ctx->d_midx.as<int>(), ctx->d_moff.as<int>(),
                                   ctx->d_tmp.as<int>(), ctx->d_out_col.as<int>(), ctx->d_out_label.as<int>(),
                                   ctx->d_out_off.as<int>(), ctx->d_bp_pts.as<int>() + ctx->bp_nnz);
            }
            // the kept masks' (col, label, off) and the 8 per-candidate statistics arrays: packed on
            // the device, one copy into pinned memory
            const size_t npack = 3 * static_cast<size_t>(Mb) + 8 * static_cast<size_t>(NS);
            ctx->d_bppack.reserve((npack + 1) * 4);
            if (ctx->h_bppack_n < npack) {
                if (ctx->h_bppack) MC_HIP(hipHostFree(ctx->h_bppack));
                ctx->h_bppack = nullptr;
                ctx->h_bppack_n = 0;
                const size_t n = npack + npack / 2 + 1024;
                MC_HIP(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_bppack), n * 4, hipHostMallocDefault));
                ctx->h_bppack_n = n;
            }
            if (npack) {
                hipLaunchKernelGGL(mc::k_bp_pack, grid_for(static_cast<int64_t>(npack)), dim3(256), 0, s, st + BS_NS, st + BS_M,
                                   ctx->d_out_col.as<int>(), ctx->d_out_label.as<int>(), ctx->d_out_off.as<int>(),
                                   ctx->d_slot_frame.as<int>(), ctx->d_slot_id.as<int>(), ctx->d_slot_np.as<int>(),
                                   ctx->d_slot_nv.as<int>(), ctx->d_slot_m.as<int>(), ctx->d_slot_ns.as<int>(),
                                   ctx->d_slot_cov.as<int>(), ctx->d_slot_nn.as<int>(), ctx->d_bppack.as<int>());
                MC_HIP(hipMemcpyAsync(ctx->h_bppack, ctx->d_bppack.ptr, npack * 4, hipMemcpyDeviceToHost, s));
            }
            MC_HIP(hipEventRecord(ctx->ev_pack, s));
            bp_debug_sync(s, "bp_emit");
            pend.valid = true;
            pend.b0 = b0;
            pend.Mb = Mb;
            pend.NS = NS;
            pend.nnzb = nnzb;
            pend.nnz_base = ctx->bp_nnz;
            ctx->bp_nnz += nnzb;
            b0 += fb;
        }
        // the next call's batches are sized for the share seen, decaying from the larger of earlier calls
        // (a stream of scenes on one context: a sparse scene does not at once size batches a denser one
        // after it overflows)
        if (mfrac_seen > 0.0) {
            ctx->bp_mfrac = ctx->bp_mfrac_obs ? std::max(mfrac_seen, 0.5 * (ctx->bp_mfrac + mfrac_seen)) : mfrac_seen;
            ctx->bp_mfrac_obs = true;
        }
        ctx->bp_last_fb = FB;
        unpack();
        MC_HIP(hipStreamSynchronize(s));
        ctx->have_bp = true;
    });
}

int mc_backproject_get_info(mc_ctx *ctx, mc_bp_info *info)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(info, MC_ERR_INVALID, "null info");
        info->num_frames = ctx->bp_F;
        info->num_candidates = static_cast<int32_t>(ctx->bp_stats.size() / MC_BP_NSTAT);
        info->num_masks = static_cast<int32_t>(ctx->bp_col.size());
        info->error_frame = ctx->bp_err_frame;
        info->num_mask_points = ctx->bp_nnz;
    });
}

int mc_backproject_get_batching(mc_ctx *ctx, int64_t *out4)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(out4, MC_ERR_INVALID, "null output");
        out4[0] = ctx->bp_last_fb;
        out4[1] = static_cast<int64_t>(ctx->bp_px_cap);
        out4[2] = static_cast<int64_t>(ctx->bp_px_cap * kBpBytesPerMaskPixel + ctx->bp_fpx_cap * kBpBytesPerFramePixel);
        out4[3] = ctx->bp_redo;
    });
}

int mc_backproject_get_masks(mc_ctx *ctx, int32_t *mask_col, int32_t *mask_label, int64_t *mask_off,
                             int32_t *mask_pts)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_bp, MC_ERR_STATE, "no back-projection result");
        const size_t M = ctx->bp_col.size();
        if (mask_col) std::copy(ctx->bp_col.begin(), ctx->bp_col.end(), mask_col);
        if (mask_label) std::copy(ctx->bp_label.begin(), ctx->bp_label.end(), mask_label);
        if (mask_off) std::copy(ctx->bp_off.begin(), ctx->bp_off.begin() + M + 1, mask_off);
        if (mask_pts && ctx->bp_nnz)
            MC_HIP(hipMemcpyAsync(mask_pts, ctx->d_bp_pts.ptr, ctx->bp_nnz * 4, hipMemcpyDeviceToHost, ctx->stream));
        MC_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int mc_backproject_copy_points_device(mc_ctx *ctx, int32_t *mask_pts_dev)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_bp, MC_ERR_STATE, "no back-projection result");
        MC_REQUIRE(mask_pts_dev || !ctx->bp_nnz, MC_ERR_INVALID, "null destination");
        if (ctx->bp_nnz)
            MC_HIP(hipMemcpyAsync(mask_pts_dev, ctx->d_bp_pts.ptr, ctx->bp_nnz * 4, hipMemcpyDeviceToDevice, ctx->stream));
    });
}

int mc_backproject_get_candidates(mc_ctx *ctx, int32_t *stats)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_bp, MC_ERR_STATE, "no back-projection result");
        std::copy(ctx->bp_stats.begin(), ctx->bp_stats.end(), stats);
    });
}

#ifdef MC_BP_STAMPS
// diagnostic builds only: read (and clear) k_bp_denoise's per-step clock totals
int mc_debug_bp_slot_times(unsigned *out, int n)
{
    n = std::min(n, 1 << 16);
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mc::g_bp_slot_time), n * 4) == hipSuccess ? MC_OK : MC_ERR_HIP;
}
int mc_debug_bp_stamps(unsigned long long *out32)
{
    if (hipMemcpyFromSymbol(out32, HIP_SYMBOL(mc::g_bp_stamps), 48 * 8) != hipSuccess) return MC_ERR_HIP;
    static const unsigned long long zero[48] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(mc::g_bp_stamps), zero, 48 * 8) == hipSuccess ? MC_OK : MC_ERR_HIP;
}
#endif

int mc_scene_use_backprojection(mc_ctx *ctx)
{
    if (!ctx) return MC_ERR_INVALID;
    if (!ctx->have_bp) {
        ctx->err = "no back-projection result";
        return MC_ERR_STATE;
    }
    const std::vector<int32_t> col = ctx->bp_col, lab = ctx->bp_label;
    const std::vector<int64_t> off = ctx->bp_off;
    return mc_scene_set_masks(ctx, ctx->P_scene, ctx->bp_F, static_cast<int32_t>(col.size()), col.data(), lab.data(),
                              off.data(), ctx->d_bp_pts.as<int32_t>(), 1);
}


// ---------------------------------------------------------------------------------------------
// post-processing (utils/post_process.py:173-194)
// ---------------------------------------------------------------------------------------------
int mc_pp_run(mc_ctx *ctx, const mc_pp_params *params, int64_t num_points, int32_t num_frames, const double *scene_xyz,
              const uint64_t *pfm_bits, int32_t num_masks, const int64_t *mask_off, const int32_t *mask_pts,
              int32_t num_nodes, const uint64_t *node_vf_bits, const int64_t *node_pt_off, const int32_t *node_pts,
              const int64_t *node_mask_off, const int32_t *node_masks, const int32_t *node_mask_col)
{
    return guarded(ctx, [&] {
        ctx->have_pp = false;
        MC_REQUIRE(params, MC_ERR_INVALID, "null params");
        MC_REQUIRE(num_points >= 0 && num_points < (1ll << 31) && num_frames >= 0 && num_masks >= 0 && num_nodes >= 0,
                   MC_ERR_INVALID, "bad sizes");
        MC_REQUIRE(num_frames <= 16384, MC_ERR_UNSUPPORTED, "num_frames must be <= 16384");
        MC_REQUIRE(params->dbscan_eps > 0 && params->dbscan_min_points >= 1, MC_ERR_INVALID, "bad DBSCAN parameters");
        MC_REQUIRE(mask_off && node_pt_off && node_mask_off, MC_ERR_INVALID, "null offsets");
        const int N = num_nodes, F = num_frames, FW = (F + 63) / 64, Mt = num_masks;
        const int64_t P = num_points, E = node_pt_off[N], Q = node_mask_off[N], MP = mask_off[Mt];
        MC_REQUIRE(node_pt_off[0] == 0 && node_mask_off[0] == 0 && mask_off[0] == 0, MC_ERR_INVALID, "offsets must start at 0");
        MC_REQUIRE(E < (1ll << 30) && Q < (1ll << 31), MC_ERR_UNSUPPORTED, "too many node points");
        MC_REQUIRE((P == 0 || (scene_xyz && pfm_bits)) && (E == 0 || node_pts) && (Q == 0 || (node_masks && node_mask_col)) &&
                       (MP == 0 || mask_pts) && (N == 0 || node_vf_bits),
                   MC_ERR_INVALID, "null argument");
        // host checks and per-node layout: the frame position of each node mask among the node's
        // visible frames (post_process.py:69), hit-bit words per node point
        std::vector<int32_t> qfpos(static_cast<size_t>(Q));
        std::vector<int64_t> hit_off(N + 1, 0);
        std::vector<int32_t> order(N);
        for (int k = 0; k < N; k++) {
            const uint64_t *vf = node_vf_bits + static_cast<int64_t>(k) * FW;
            int nvf = 0;
            for (int w = 0; w < FW; w++) nvf += __builtin_popcountll(vf[w]);
            const int64_t n = node_pt_off[k + 1] - node_pt_off[k];
            MC_REQUIRE(n >= 0 && node_mask_off[k + 1] >= node_mask_off[k], MC_ERR_INVALID, "offsets must be ascending");
            for (int64_t q = node_mask_off[k]; q < node_mask_off[k + 1]; q++) {
                const int c = node_mask_col[q], m = node_masks[q];
                MC_REQUIRE(m >= 0 && m < Mt, MC_ERR_INVALID, "node mask index out of range");
                MC_REQUIRE(c >= 0 && c < F && ((vf[c >> 6] >> (c & 63)) & 1ull), MC_ERR_INVALID,
                           "a mask's frame is not among the node's visible frames (post_process.py:69 IndexError)");
                int pos = 0;
                for (int w = 0; w < (c >> 6); w++) pos += __builtin_popcountll(vf[w]);
                pos += __builtin_popcountll(vf[c >> 6] & ((1ull << (c & 63)) - 1));
                qfpos[q] = pos;
            }
            hit_off[k + 1] = hit_off[k] + n * ((nvf + 63) / 64);
            order[k] = k;
        }
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
            return node_pt_off[a + 1] - node_pt_off[a] > node_pt_off[b + 1] - node_pt_off[b];
        });
        for (int64_t i = 0; i < E; i++) MC_REQUIRE(node_pts[i] >= 0 && node_pts[i] < P, MC_ERR_INVALID, "node point out of range");
        {  // the DBSCAN grid packs cell coordinates in 21 bits per axis (pack3): every node's extent
           // must stay below 2^21 cells of 1.01 eps, or neighbours would be missed silently
            const double ce = params->dbscan_eps * 1.01;
            for (int k = 0; k < N; k++) {
                double mn[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, mx[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
                for (int64_t i = node_pt_off[k]; i < node_pt_off[k + 1]; i++)
                    for (int c = 0; c < 3; c++) {
                        const double v = scene_xyz[3 * static_cast<int64_t>(node_pts[i]) + c];
                        mn[c] = std::min(mn[c], v);
                        mx[c] = std::max(mx[c], v);
                    }
                for (int c = 0; c < 3; c++)
                    MC_REQUIRE(!(mx[c] >= mn[c]) || std::floor((mx[c] - mn[c]) / ce) < double((1 << 21) - 1),
                               MC_ERR_UNSUPPORTED, "a node spans more than 2^21 DBSCAN cells per axis (eps too small)");
            }
        }
        for (int64_t i = 0; i < MP; i++) MC_REQUIRE(mask_pts[i] >= 0 && mask_pts[i] < P, MC_ERR_INVALID, "mask point out of range");

        hipStream_t s = ctx->stream;
        auto up = [&](DevBuf &b, const void *h, size_t bytes) {
            b.reserve(bytes + 8);
            if (bytes) MC_HIP(hipMemcpyAsync(b.ptr, h, bytes, hipMemcpyHostToDevice, s));
        };
        DevBuf scene, pfm, moff, mpts, npoff, npts, nvf, qoff, qm, qfp, hoff, dorder;
        up(scene, scene_xyz, static_cast<size_t>(P) * 24);
        up(pfm, pfm_bits, static_cast<size_t>(P) * FW * 8);
        up(moff, mask_off, static_cast<size_t>(Mt + 1) * 8);
        up(mpts, mask_pts, static_cast<size_t>(MP) * 4);
        up(npoff, node_pt_off, static_cast<size_t>(N + 1) * 8);
        up(npts, node_pts, static_cast<size_t>(E) * 4);
        up(nvf, node_vf_bits, static_cast<size_t>(N) * FW * 8);
        up(qoff, node_mask_off, static_cast<size_t>(N + 1) * 8);
        up(qm, node_masks, static_cast<size_t>(Q) * 4);
        up(qfp, qfpos.data(), static_cast<size_t>(Q) * 4);
        up(hoff, hit_off.data(), static_cast<size_t>(N + 1) * 8);
        up(dorder, order.data(), static_cast<size_t>(N) * 4);

        mc::PPDev pr;
        pr.eps2 = params->dbscan_eps * params->dbscan_eps;
        pr.ce = params->dbscan_eps * 1.01;
        pr.thr = params->point_filter_threshold;
        pr.ratio = params->overlapping_ratio;
        pr.minpts = params->dbscan_min_points;

        // ---- DBSCAN split (dbscan_process) ----
        DevBuf xyz, pcell, pbkt, bcnt, bstart, blist, ncnt, par, root, rnk, lab, ccnt, nob, nsh, tick, skey, sxyz, sidx;
        skey.reserve(E * 8 + 8);  // bucket-ordered copies of the cell keys, points and indices
        sxyz.reserve(E * 24 + 8);
        sidx.reserve(E * 4 + 8);
        xyz.reserve(E * 24 + 8);
        pcell.reserve(E * 8 + 8);
        for (DevBuf *b : {&pbkt, &blist, &ncnt, &par, &root, &rnk, &lab}) b->reserve(E * 4 + 8);
        bcnt.reserve((2 * E + N + 1) * 4);
        bstart.reserve((2 * E + N + 1) * 4);
        ccnt.reserve((E + N + 1) * 4);
        nob.reserve(N * 4 + 8);
        nsh.reserve(N * 4 + 8);
        tick.reserve(16);
        MC_HIP(hipMemsetAsync(bcnt.ptr, 0, (2 * E + N + 1) * 4, s));
        MC_HIP(hipMemsetAsync(tick.ptr, 0, 16, s));
        {
            mc::TimedScope ts(ctx->timer, s, "pp_dbscan");
            if (E) hipLaunchKernelGGL(mc::k_pp_gather, grid_for(3 * E), dim3(256), 0, s, scene.as<double>(), npts.as<int>(), E,
                                      xyz.as<double>());
            // nodes above big_min points (the first nbig of the size order) are split over the chip
            int big_min = mc::kPPLdsUF;
            if (const char *e = getenv("MC_PP_BIG_MIN")) big_min = std::max(1, atoi(e));
            int nbig = 0;
            std::vector<int2> items;
            while (nbig < N && node_pt_off[order[nbig] + 1] - node_pt_off[order[nbig]] > big_min) {
                const int k = order[nbig++];
                const int n = static_cast<int>(node_pt_off[k + 1] - node_pt_off[k]);
                for (int c = 0; c < n; c += 512) items.push_back(make_int2(k, c));
            }
            if (nbig) {
                DevBuf ditems, gcm;
                up(ditems, items.data(), items.size() * sizeof(int2));
                gcm.reserve(static_cast<size_t>(N) * 12 + 8);
                const mc::PPBig b{npoff.as<int64_t>(), xyz.as<double>(), pcell.as<unsigned long long>(), pbkt.as<int>(),
                                  bcnt.as<int>(), bstart.as<int>(), blist.as<int>(), ncnt.as<int>(), par.as<int>(),
                                  root.as<int>(), rnk.as<int>(), lab.as<int>(), ccnt.as<int>(), gcm.as<int>()};
                const int ni = static_cast<int>(items.size());
                hipLaunchKernelGGL(mc::k_pp_big_grid<512>, dim3(nbig), dim3(512), 0, s, nbig, dorder.as<int>(), pr, b);
                hipLaunchKernelGGL((mc::k_pp_big_walk<512, 0>), dim3(std::min(ni, 65536)), dim3(512), 0, s, ni,
                                   ditems.as<int2>(), pr, b);
                hipLaunchKernelGGL((mc::k_pp_big_walk<512, 1>), dim3(std::min(ni, 65536)), dim3(512), 0, s, ni,
                                   ditems.as<int2>(), pr, b);
                hipLaunchKernelGGL(mc::k_pp_big_label<512>, dim3(nbig), dim3(512), 0, s, nbig, dorder.as<int>(), pr, b,
                                   nob.as<int>(), nsh.as<int>());
                MC_HIP(hipGetLastError());
                MC_HIP(hipStreamSynchronize(s));  // ditems / gcm are freed at scope exit
            }
            if (N > nbig)  // 512-thread workgroups (1024 spills the neighbour walks)
                hipLaunchKernelGGL(mc::k_pp_dbscan<512>, dim3(std::max(1, std::min(N - nbig, ctx->num_cu * 2))), dim3(512), 0, s,
                                   N - nbig, dorder.as<int>() + nbig, tick.as<int>(),
                                      npoff.as<int64_t>(), pr, xyz.as<double>(), pcell.as<unsigned long long>(), pbkt.as<int>(),
                                      bcnt.as<int>(), bstart.as<int>(), blist.as<int>(), ncnt.as<int>(), par.as<int>(),
                                      root.as<int>(), rnk.as<int>(), lab.as<int>(), ccnt.as<int>(), nob.as<int>(), nsh.as<int>(),
                                      skey.as<unsigned long long>(), sxyz.as<double>(), sidx.as<int>());
            MC_HIP(hipGetLastError());
        }
        std::vector<int32_t> h_nob(N), h_base(N + 1, 0);
        if (N) MC_HIP(hipMemcpyAsync(h_nob.data(), nob.ptr, N * 4, hipMemcpyDeviceToHost, s));
        MC_HIP(hipStreamSynchronize(s));
        for (int k = 0; k < N; k++) h_base[k + 1] = h_base[k] + h_nob[k];
        const int K = h_base[N];
        DevBuf obase;
        up(obase, h_base.data(), static_cast<size_t>(N + 1) * 4);

        // ---- filter_point ----
        const int slots = std::max(1, std::min(N, ctx->num_cu));
        if (ctx->pp_posmap_P < P || ctx->pp_posmap_slots < slots) {
            ctx->d_pp_posmap.release();
            ctx->d_pp_posmap.reserve(static_cast<size_t>(slots) * P * 4 + 8);
            MC_HIP(hipMemsetAsync(ctx->d_pp_posmap.ptr, 0xFF, static_cast<size_t>(slots) * P * 4, s));
            ctx->pp_posmap_P = P;
            ctx->pp_posmap_slots = slots;
        }
        const int64_t H = hit_off[N];
        DevBuf hit, cvid, qobj, qcov, onm, onv, obox, eobj;
        hit.reserve(H * 8 + 8);
        cvid.reserve(E * 4 + 8);
        qobj.reserve(Q * 4 + 8);
        qcov.reserve(Q * 8 + 8);
        onm.reserve(K * 4 + 8);
        onv.reserve(K * 4 + 8);
        obox.reserve(K * 48 + 8);
        eobj.reserve(E * 4 + 8);
        if (H) MC_HIP(hipMemsetAsync(hit.ptr, 0, H * 8, s));
        if (K) MC_HIP(hipMemsetAsync(onm.ptr, 0, K * 4, s));
        {
            mc::TimedScope ts(ctx->timer, s, "pp_filter");
            if (N) hipLaunchKernelGGL(mc::k_pp_filter, dim3(slots), dim3(256), 0, s, N, dorder.as<int>(), tick.as<int>() + 1, pr,
                                      FW, P, npoff.as<int64_t>(), npts.as<int>(), nvf.as<unsigned long long>(),
                                      hoff.as<int64_t>(), qoff.as<int64_t>(), qm.as<int>(), qfp.as<int>(), moff.as<int64_t>(),
                                      mpts.as<int>(), pfm.as<unsigned long long>(), xyz.as<double>(), lab.as<int>(),
                                      ccnt.as<int>(), nob.as<int>(), nsh.as<int>(), obase.as<int>(), ctx->d_pp_posmap.as<int>(),
                                      hit.as<unsigned long long>(), cvid.as<int>(), qobj.as<int>(), qcov.as<double>(),
                                      onm.as<int>(), onv.as<int>(), obox.as<double>(), eobj.as<int>());
            MC_HIP(hipGetLastError());
        }
        std::vector<int32_t> h_nm(K), h_nv(K);
        std::vector<double> h_box(static_cast<size_t>(K) * 6);
        if (K) {
            MC_HIP(hipMemcpyAsync(h_nm.data(), onm.ptr, K * 4, hipMemcpyDeviceToHost, s));
            MC_HIP(hipMemcpyAsync(h_nv.data(), onv.ptr, K * 4, hipMemcpyDeviceToHost, s));
            MC_HIP(hipMemcpyAsync(h_box.data(), obox.ptr, K * 48, hipMemcpyDeviceToHost, s));
        }
        MC_HIP(hipStreamSynchronize(s));
        // objects kept by filter_point (:96): a kept point and >= 2 masks
        std::vector<int32_t> kidx(K, -1), kept;
        std::vector<double> kbox;
        std::vector<int32_t> klen;
        for (int o = 0; o < K; o++)
            if (h_nv[o] > 0 && h_nm[o] >= 2) {
                kidx[o] = static_cast<int32_t>(kept.size());
                kept.push_back(o);
                kbox.insert(kbox.end(), h_box.begin() + 6 * o, h_box.begin() + 6 * o + 6);
                klen.push_back(h_nv[o]);
            }
        const int Kk = static_cast<int>(kept.size());
        MC_REQUIRE(Kk <= 46340, MC_ERR_UNSUPPORTED, "more than 46340 objects after filter_point");

        // ---- merge_overlapping_objects ----
        std::vector<uint8_t> h_inv(Kk, 0);
        if (Kk > 1) {
            mc::TimedScope ts(ctx->timer, s, "pp_merge");
            DevBuf dk, pcnt, plist, mxc, inter, dbox, dlen, dec, inv;
            up(dk, kidx.data(), static_cast<size_t>(K) * 4);
            up(dbox, kbox.data(), static_cast<size_t>(Kk) * 48);
            up(dlen, klen.data(), static_cast<size_t>(Kk) * 4);
            pcnt.reserve(P * 4 + 8);
            mxc.reserve(8);
            int sl = mc::kPPSlots;
            for (int pass = 0; pass < 2; pass++) {
                plist.reserve(static_cast<size_t>(P) * sl * 4 + 8);
                MC_HIP(hipMemsetAsync(pcnt.ptr, 0, P * 4, s));
                MC_HIP(hipMemsetAsync(mxc.ptr, 0, 4, s));
                hipLaunchKernelGGL(mc::k_pp_index, grid_for(E), dim3(256), 0, s, E, npts.as<int>(), eobj.as<int>(), dk.as<int>(),
                                   sl, pcnt.as<int>(), plist.as<int>(), mxc.as<int>());
                int mx = 0;
                MC_HIP(hipMemcpyAsync(&mx, mxc.ptr, 4, hipMemcpyDeviceToHost, s));
                MC_HIP(hipStreamSynchronize(s));
                if (mx <= sl) break;
                sl = mx;
            }
            inter.reserve(static_cast<size_t>(Kk) * Kk * 4);
            dec.reserve(static_cast<size_t>(Kk) * Kk);
            inv.reserve(Kk + 8);
            MC_HIP(hipMemsetAsync(inter.ptr, 0, static_cast<size_t>(Kk) * Kk * 4, s));
            hipLaunchKernelGGL(mc::k_pp_pairs, grid_for(P), dim3(256), 0, s, P, sl, pcnt.as<int>(), plist.as<int>(), Kk,
                               inter.as<int>());
            int kCap = 1 << 16;  // non-zero decisions handled by the host pass; more: k_pp_greedy
            if (const char *e = getenv("MC_PP_GREEDY_CAP")) kCap = std::max(0, atoi(e));  // tests force the device pass
            DevBuf nl, lst;
            nl.reserve(8);
            lst.reserve(static_cast<size_t>(std::max(kCap, 1)) * sizeof(int2));
            MC_HIP(hipMemsetAsync(nl.ptr, 0, 4, s));
            hipLaunchKernelGGL(mc::k_pp_decide, grid_for(static_cast<int64_t>(Kk) * Kk), dim3(256), 0, s, Kk, pr,
                               dbox.as<double>(), dlen.as<int>(), inter.as<int>(), dec.as<unsigned char>(), kCap,
                               nl.as<int>(), lst.as<int2>());
            MC_HIP(hipGetLastError());
            int nd = 0;
            MC_HIP(hipMemcpyAsync(&nd, nl.ptr, 4, hipMemcpyDeviceToHost, s));
            MC_HIP(hipStreamSynchronize(s));
            if (nd <= kCap) {
                // the greedy pass (post_process.py:14-29) over the non-zero decisions only: zero
                // decisions change nothing, so visiting (i, j) ascending is the reference's loop
                std::vector<int2> d(nd);
                if (nd) MC_HIP(hipMemcpy(d.data(), lst.ptr, static_cast<size_t>(nd) * sizeof(int2), hipMemcpyDeviceToHost));
                auto jj = [](const int2 &v) { return v.y < 0 ? -1 - v.y : v.y; };
                std::sort(d.begin(), d.end(), [&](const int2 &a, const int2 &b) {
                    return a.x != b.x ? a.x < b.x : jj(a) < jj(b);
                });
                int row = -1;
                bool skip = false;
                for (const int2 &v : d) {
                    if (v.x != row) {  // "if invalid_object[i]: continue" is read once per row (:15)
                        row = v.x;
                        skip = h_inv[row] != 0;
                    }
                    if (skip || h_inv[jj(v)]) continue;
                    if (v.y < 0) h_inv[v.x] = 1;
                    else h_inv[v.y] = 1;
                }
            } else {
                hipLaunchKernelGGL(mc::k_pp_greedy, dim3(1), dim3(1024), 0, s, Kk, dec.as<unsigned char>(), inv.as<unsigned char>());
                MC_HIP(hipGetLastError());
                MC_HIP(hipMemcpyAsync(h_inv.data(), inv.ptr, Kk, hipMemcpyDeviceToHost, s));
                MC_HIP(hipStreamSynchronize(s));  // h_inv is pageable host memory read just below
            }
        }
        // ---- results ----
        ctx->pp_state.assign(K, 0);
        int nfin = 0;
        for (int i = 0; i < Kk; i++) {
            ctx->pp_state[kept[i]] = h_inv[i] ? 1 : 2;
            nfin += h_inv[i] ? 0 : 1;
        }
        ctx->pp_entry_obj.resize(E);
        ctx->pp_qobj.resize(Q);
        ctx->pp_qcov.resize(Q);
        if (E) MC_HIP(hipMemcpyAsync(ctx->pp_entry_obj.data(), eobj.ptr, E * 4, hipMemcpyDeviceToHost, s));
        if (Q) {
            MC_HIP(hipMemcpyAsync(ctx->pp_qobj.data(), qobj.ptr, Q * 4, hipMemcpyDeviceToHost, s));
            MC_HIP(hipMemcpyAsync(ctx->pp_qcov.data(), qcov.ptr, Q * 8, hipMemcpyDeviceToHost, s));
        }
        MC_HIP(hipStreamSynchronize(s));
        ctx->timer.collect();
        for (auto &o : ctx->pp_entry_obj)
            if (o >= 0 && ctx->pp_state[o] != 2) o = -1;
        ctx->pp_obj_node.resize(K);
        for (int k = 0; k < N; k++)
            for (int o = h_base[k]; o < h_base[k + 1]; o++) ctx->pp_obj_node[o] = k;
        ctx->pp_box = std::move(h_box);
        ctx->pp_info.num_objects = K;
        ctx->pp_info.num_filtered = Kk;
        ctx->pp_info.num_final = nfin;
        ctx->pp_info.num_entries = E;
        ctx->pp_info.num_node_masks = Q;
        ctx->have_pp = true;
    });
}

int mc_pp_get_info(mc_ctx *ctx, mc_pp_info *info)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_pp, MC_ERR_STATE, "no post-processing result");
        MC_REQUIRE(info, MC_ERR_INVALID, "null argument");
        *info = ctx->pp_info;
    });
}

int mc_pp_get_results(mc_ctx *ctx, int32_t *entry_object, int32_t *mask_object, double *mask_coverage,
                      uint8_t *object_state, int32_t *object_node, double *object_bbox)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(ctx->have_pp, MC_ERR_STATE, "no post-processing result");
        auto cp = [](void *dst, const void *src, size_t bytes) {
            if (dst && bytes) std::memcpy(dst, src, bytes);
        };
        cp(entry_object, ctx->pp_entry_obj.data(), ctx->pp_entry_obj.size() * 4);
        cp(mask_object, ctx->pp_qobj.data(), ctx->pp_qobj.size() * 4);
        cp(mask_coverage, ctx->pp_qcov.data(), ctx->pp_qcov.size() * 8);
        cp(object_state, ctx->pp_state.data(), ctx->pp_state.size());
        cp(object_node, ctx->pp_obj_node.data(), ctx->pp_obj_node.size() * 4);
        cp(object_bbox, ctx->pp_box.data(), ctx->pp_box.size() * 8);
    });
}


// ---------------------------------------------------------------------------------------------
// instance-evaluation match counts (evaluation/evaluate.py:254-329)
// ---------------------------------------------------------------------------------------------
int mc_eval_match_counts(mc_ctx *ctx, int64_t num_points, int32_t num_pred, const uint8_t *pred_masks,
                         const int32_t *gt_instance, int32_t num_gt, const uint8_t *void_flags, int64_t *pred_verts,
                         int64_t *void_intersection, int64_t *intersection)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(num_points >= 0 && num_pred >= 0 && num_gt >= 0, MC_ERR_INVALID, "negative size");
        MC_REQUIRE((num_points == 0 || (gt_instance && void_flags && (num_pred == 0 || pred_masks))) &&
                       (num_pred == 0 || (pred_verts && void_intersection && (num_gt == 0 || intersection))),
                   MC_ERR_INVALID, "null argument");
        const int64_t P = num_points;
        const int K = num_pred, G = num_gt;
        for (int64_t p = 0; p < P; p++)
            MC_REQUIRE(gt_instance[p] >= -1 && gt_instance[p] < G, MC_ERR_INVALID, "gt instance index out of range");
        hipStream_t s = ctx->stream;
        DevBuf dpred, dg, dv, dverts, dvi, dint;
        dpred.reserve(static_cast<size_t>(P) * K + 8);
        dg.reserve(P * 4 + 8);
        dv.reserve(P + 8);
        dverts.reserve(K * 8 + 8);
        dvi.reserve(K * 8 + 8);
        dint.reserve(static_cast<size_t>(K) * G * 8 + 8);
        if (P && K) MC_HIP(hipMemcpyAsync(dpred.ptr, pred_masks, static_cast<size_t>(P) * K, hipMemcpyHostToDevice, s));
        if (P) {
            MC_HIP(hipMemcpyAsync(dg.ptr, gt_instance, P * 4, hipMemcpyHostToDevice, s));
            MC_HIP(hipMemcpyAsync(dv.ptr, void_flags, P, hipMemcpyHostToDevice, s));
        }
        MC_HIP(hipMemsetAsync(dverts.ptr, 0, K * 8 + 8, s));
        MC_HIP(hipMemsetAsync(dvi.ptr, 0, K * 8 + 8, s));
        MC_HIP(hipMemsetAsync(dint.ptr, 0, static_cast<size_t>(K) * G * 8 + 8, s));
        {
            mc::TimedScope ts(ctx->timer, s, "eval_counts");
            if (P && K)
                hipLaunchKernelGGL(mc::k_eval_counts, grid_for(P, 256, 8192), dim3(256), 0, s, P, K, G, dpred.as<unsigned char>(),
                                   dg.as<int>(), dv.as<unsigned char>(), dverts.as<unsigned long long>(),
                                   dvi.as<unsigned long long>(), dint.as<unsigned long long>());
            MC_HIP(hipGetLastError());
        }
        if (K) {
            MC_HIP(hipMemcpyAsync(pred_verts, dverts.ptr, K * 8, hipMemcpyDeviceToHost, s));
            MC_HIP(hipMemcpyAsync(void_intersection, dvi.ptr, K * 8, hipMemcpyDeviceToHost, s));
            if (G) MC_HIP(hipMemcpyAsync(intersection, dint.ptr, static_cast<size_t>(K) * G * 8, hipMemcpyDeviceToHost, s));
        }
        MC_HIP(hipStreamSynchronize(s));
        ctx->timer.collect();
    });
}


// ---------------------------------------------------------------------------------------------
// frame decode (dataset/scannet.py:49-54, :68-73)
// ---------------------------------------------------------------------------------------------
int mc_frames_decode(mc_ctx *ctx, int32_t num_frames, int32_t height, int32_t width, const uint16_t *depth,
                     double depth_scale, int32_t seg_height, int32_t seg_width, const uint8_t *seg, int inputs_on_device,
                     float *depth_out, uint8_t *seg_out)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(num_frames >= 0 && height >= 0 && width >= 0 && seg_height >= 0 && seg_width >= 0, MC_ERR_INVALID,
                   "negative size");
        MC_REQUIRE((!depth || (depth_out && depth_scale != 0.0)) && (!seg || (seg_out && seg_height > 0 && seg_width > 0)),
                   MC_ERR_INVALID, "missing output or bad scale");
        const int64_t total = static_cast<int64_t>(num_frames) * height * width;
        const int64_t stotal = static_cast<int64_t>(num_frames) * seg_height * seg_width;
        // cv2.resize(..., INTER_NEAREST) tables (OpenCV resizeNN): src = min(floor(dst * (1 / (dsize / ssize))), ssize - 1)
        std::vector<int> yo(std::max(height, 1)), xo(std::max(width, 1));
        const double ify = 1.0 / (static_cast<double>(height) / seg_height), ifx = 1.0 / (static_cast<double>(width) / seg_width);
        for (int y = 0; y < height; y++) yo[y] = std::min(static_cast<int>(std::floor(y * ify)), seg_height - 1);
        for (int x = 0; x < width; x++) xo[x] = std::min(static_cast<int>(std::floor(x * ifx)), seg_width - 1);
        hipStream_t s = ctx->stream;
        DevBuf dd, ds, dyo, dxo;
        const unsigned short *din = reinterpret_cast<const unsigned short *>(depth);
        const unsigned char *sin = seg;
        if (!inputs_on_device) {
            if (depth) {
                dd.reserve(total * 2 + 8);
                if (total) MC_HIP(hipMemcpyAsync(dd.ptr, depth, total * 2, hipMemcpyHostToDevice, s));
                din = dd.as<unsigned short>();
            }
            if (seg) {
                ds.reserve(stotal + 8);
                if (stotal) MC_HIP(hipMemcpyAsync(ds.ptr, seg, stotal, hipMemcpyHostToDevice, s));
                sin = ds.as<unsigned char>();
            }
        }
        dyo.reserve(yo.size() * 4);
        dxo.reserve(xo.size() * 4);
        MC_HIP(hipMemcpyAsync(dyo.ptr, yo.data(), yo.size() * 4, hipMemcpyHostToDevice, s));
        MC_HIP(hipMemcpyAsync(dxo.ptr, xo.data(), xo.size() * 4, hipMemcpyHostToDevice, s));
        {
            mc::TimedScope ts(ctx->timer, s, "frames_decode");
            if (total && (depth || seg))
                hipLaunchKernelGGL(mc::k_frames_decode, grid_for(total, 256, 16384), dim3(256), 0, s, total, height, width,
                                   seg_height, seg_width, depth ? din : nullptr, depth_scale, seg ? sin : nullptr,
                                   dyo.as<int>(), dxo.as<int>(), depth_out, seg_out);
            MC_HIP(hipGetLastError());
        }
        MC_HIP(hipStreamSynchronize(s));
        ctx->timer.collect();
    });
}

// ---------------------------------------------------------------------------------------------
// host: packed bit rows -> bool bytes (the reference's dense point_frame_matrix, construction.py:40)
// ---------------------------------------------------------------------------------------------
int mc_bits_unpack(const uint64_t *words, int64_t rows, int32_t words_per_row, int32_t ncols, uint8_t *out)
{
    if (rows < 0 || words_per_row < 0 || ncols < 0 || static_cast<int64_t>(ncols) > 64ll * words_per_row)
        return MC_ERR_INVALID;
    if (!rows || !ncols) return MC_OK;
    if (!words || !out) return MC_ERR_INVALID;
    static const auto lut = [] {  // byte value -> its 8 bits as 8 bytes (little-endian)
        std::vector<uint64_t> t(256);
        for (int v = 0; v < 256; v++) {
            uint64_t x = 0;
            for (int b = 0; b < 8; b++) x |= static_cast<uint64_t>((v >> b) & 1) << (8 * b);
            t[v] = x;
        }
        return t;
    }();
    auto work = [&](int64_t r0, int64_t r1) {
        const int full = ncols / 8;  // whole output bytes groups of 8 columns
        for (int64_t r = r0; r < r1; r++) {
            const uint8_t *wb = reinterpret_cast<const uint8_t *>(words + r * words_per_row);
            uint8_t *o = out + r * ncols;
            for (int j = 0; j < full; j++) {
                const uint64_t x = lut[wb[j]];
                memcpy(o + 8 * j, &x, 8);
            }
            for (int c = 8 * full; c < ncols; c++) o[c] = static_cast<uint8_t>((wb[c >> 3] >> (c & 7)) & 1u);
        }
    };
    const int64_t bytes = rows * ncols;
    int nt = static_cast<int>(std::min<int64_t>(std::min(8u, std::max(1u, std::thread::hardware_concurrency())),
                                                std::max<int64_t>(1, bytes >> 22)));
    if (const char *e = getenv("MC_STAGE_THREADS")) nt = std::max(1, std::min(64, atoi(e)));
    if (nt <= 1) {
        work(0, rows);
        return MC_OK;
    }
    std::vector<std::thread> th;
    const int64_t step = (rows + nt - 1) / nt;
    for (int t = 1; t < nt; t++) th.emplace_back(work, std::min(rows, t * step), std::min(rows, (t + 1) * step));
    work(0, std::min(rows, step));
    for (auto &x : th) x.join();
    return MC_OK;
}

// ---------------------------------------------------------------------------------------------
// open-vocabulary label query
// ---------------------------------------------------------------------------------------------
int mc_openvoc_query(mc_ctx *ctx, int32_t num_objects, const int64_t *obj_off, const int32_t *obj_rows,
                     int32_t num_rows, int32_t dim, const float *features, int32_t num_labels,
                     const float *label_features, float temperature, int32_t *out_label)
{
    return guarded(ctx, [&] {
        MC_REQUIRE(num_objects >= 0 && num_rows >= 0 && dim > 0 && dim <= 12288 && num_labels > 0, MC_ERR_INVALID,
                   "bad sizes");
        MC_REQUIRE(obj_off && out_label && label_features && (num_rows == 0 || features), MC_ERR_INVALID, "null array");
        MC_REQUIRE(obj_off[0] == 0, MC_ERR_INVALID, "obj_off[0] != 0");
        const int64_t nr = obj_off[num_objects];
        MC_REQUIRE(nr == 0 || obj_rows, MC_ERR_INVALID, "null array");
        for (int k = 0; k < num_objects; k++) MC_REQUIRE(obj_off[k + 1] >= obj_off[k], MC_ERR_INVALID, "obj_off not ascending");
        for (int64_t i = 0; i < nr; i++)
            MC_REQUIRE(obj_rows[i] >= 0 && obj_rows[i] < num_rows, MC_ERR_INVALID, "feature row out of range");
        if (!num_objects) return;
        hipStream_t s = ctx->stream;
        DevBuf doff, drows, dfeat, dlab, dsim, dout;
        doff.reserve((num_objects + 1) * 8);
        drows.reserve((nr + 1) * 4);
        dfeat.reserve(static_cast<size_t>(num_rows) * dim * 4 + 4);
        dlab.reserve(static_cast<size_t>(num_labels) * dim * 4);
        dsim.reserve(static_cast<size_t>(num_objects) * num_labels * 4);
        dout.reserve(static_cast<size_t>(num_objects) * 4);
        MC_HIP(hipMemcpyAsync(doff.ptr, obj_off, (num_objects + 1) * 8, hipMemcpyHostToDevice, s));
        if (nr) MC_HIP(hipMemcpyAsync(drows.ptr, obj_rows, nr * 4, hipMemcpyHostToDevice, s));
        if (num_rows) MC_HIP(hipMemcpyAsync(dfeat.ptr, features, static_cast<size_t>(num_rows) * dim * 4, hipMemcpyHostToDevice, s));
        MC_HIP(hipMemcpyAsync(dlab.ptr, label_features, static_cast<size_t>(num_labels) * dim * 4, hipMemcpyHostToDevice, s));
        {
            TimedScope ts(ctx->timer, s, "ov_query");
            hipLaunchKernelGGL(mc::k_ov_query, dim3(num_objects), dim3(256), dim * sizeof(float), s, num_objects,
                               doff.as<long long>(), drows.as<int>(), dim, dfeat.as<float>(), num_labels,
                               dlab.as<float>(), temperature, dsim.as<float>(), dout.as<int>());
        }
        MC_HIP(hipGetLastError());
        MC_HIP(hipMemcpyAsync(out_label, dout.ptr, static_cast<size_t>(num_objects) * 4, hipMemcpyDeviceToHost, s));
        MC_HIP(hipStreamSynchronize(s));
    });
}

}  // extern "C"
