/*
 * mcgraph.h — C-ABI of the MI355X-native view-consensus graph path of
 * MaskClustering (libmcgraph.so, hand-written HIP kernels for gfx950).
 *
 * The library replaces the compute behind these reference interfaces
 * (paths relative to the reference repository):
 *
 *   graph/construction.py:7    mask_graph_construction      -> mc_scene_set_masks + mc_graph_build
 *   graph/construction.py:22   build_point_in_mask_matrix   -> mc_graph_build (S2)
 *   graph/construction.py:137  process_masks / :98 process_one_mask -> mc_graph_build (S3)
 *   graph/construction.py:80   get_observer_num_thresholds  -> mc_graph_build (S4) + mc_graph_get_thresholds
 *   graph/construction.py:66   init_nodes                   -> mc_graph_build (S5)
 *   graph/iterative_clustering.py:36 iterative_clustering   -> mc_cluster_run
 *   graph/iterative_clustering.py:13 update_graph           -> mc_cluster_run (pair counts + edge rule)
 *   graph/iterative_clustering.py:5  cluster_into_new_nodes -> mc_cluster_run (components)
 *   graph/node.py:24           Node.create_node_from_list   -> mc_cluster_run (on-device merge)
 *   utils/mask_backprojection.py:70 turn_mask_to_point      -> mc_backproject (S1)
 *   utils/mask_backprojection.py:154 frame_backprojection   -> mc_backproject + mc_backproject_get_masks
 *   utils/geometry.py:9        denoise                      -> mc_backproject (S1 denoise)
 *
 * Conventions
 *   - Every call returns 0 (MC_OK) or an MC_ERR_* code; mc_ctx_last_error()
 *     gives the message.  No call throws.
 *   - Host buffers are caller-owned; sizes are given by the *_get_info calls
 *     (two-call pattern: query sizes, then fill).
 *   - The context owns all device memory.  One context per device per host
 *     thread; no global state.  Work is enqueued on the context's HIP stream
 *     (its own, or the one given by mc_ctx_set_stream); getters synchronise it.
 *   - Masks are the reference's per-frame mask dicts flattened in frame
 *     order, ids in dict order (construction.py:46-60); frames whose mask
 *     union is empty are dropped like construction.py:50-51.
 */
#ifndef MCGRAPH_H
#define MCGRAPH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MC_OK 0
#define MC_ERR_INVALID 1          /* bad argument / inconsistent input            */
#define MC_ERR_HIP 2              /* HIP runtime error                            */
#define MC_ERR_STATE 3            /* call out of order (e.g. cluster before build)*/
#define MC_ERR_EMPTY_OBSERVERS 4  /* np.percentile on empty (construction.py:89)   */
#define MC_ERR_UNSUPPORTED 5      /* size beyond a documented limit                */
#define MC_ERR_NO_NODES 6         /* torch.stack([]) (iterative_clustering.py:17)  */

typedef struct mc_ctx mc_ctx;

/* args fields read by graph/construction.py:119,125,132 */
typedef struct {
    double mask_visible_threshold;
    double contained_threshold;
    double undersegment_filter_threshold;
} mc_graph_params;

typedef struct {
    int64_t num_points;        /* P                                   */
    int32_t num_frames;        /* F (columns of the frame list)       */
    int32_t num_masks;         /* M: global masks (kept)              */
    int32_t num_undersegment;  /* |U|                                 */
    int32_t num_nodes0;        /* N0 = M - |U|                        */
    int64_t num_contained;     /* nnz of contained_masks after undo   */
    int64_t num_boundary;      /* |boundary_points|                   */
    int32_t num_thresholds;    /* len(observer_num_thresholds)        */
    int32_t threshold_status;  /* MC_OK or MC_ERR_EMPTY_OBSERVERS     */
} mc_graph_info;

typedef struct {
    int32_t num_iterations;    /* thresholds consumed                 */
    int32_t num_objects;       /* final nodes                         */
    int32_t num_nodes0;        /* nodes entering iteration 0          */
    int32_t reserved;
    int64_t num_object_points; /* sum over objects of |point_ids|     */
    int64_t num_object_contained; /* sum over objects of |contained|  */
    int64_t num_object_masks;  /* sum over objects of |mask_list|     */
} mc_cluster_info;

/* S1 constants (utils/mask_backprojection.py:8-14,38; utils/geometry.py:10,16,22).
 * Same layout as the oracle's orc_bp_params.  mc_bp_params_default() fills
 * the reference's values. */
typedef struct {
    double depth_trunc;            /* DEPTH_TRUNC = 20                      */
    double voxel_size;             /* DISTANCE_THRESHOLD = 0.01 (voxel)     */
    double dbscan_eps;             /* 0.04                                  */
    double component_min_fraction; /* 0.2                                   */
    double sor_std_ratio;          /* 2.0                                   */
    double ball_radius;            /* DISTANCE_THRESHOLD (as float32)       */
    double coverage_threshold;     /* COVERAGE_THRESHOLD = 0.3              */
    int32_t dbscan_min_points;     /* 4                                     */
    int32_t sor_neighbors;         /* 20 (<= 20)                            */
    int32_t ball_k;                /* K = 20 (<= 32)                        */
    int32_t few_points;            /* FEW_POINTS_THRESHOLD = 25             */
} mc_bp_params;

typedef struct {
    int32_t num_frames;
    int32_t num_candidates;        /* (frame, id) with >= few_points pixels  */
    int32_t num_masks;             /* kept masks (coverage >= threshold)     */
    int32_t error_frame;           /* -1, or the first frame that raises     */
    int64_t num_mask_points;       /* sum of the kept masks' set sizes       */
} mc_bp_info;

#define MC_BP_NSTAT 10  /* per candidate: frame, id, pixels, voxels, after DBSCAN filter,
                           after outlier removal, -1, covered, neighbours, kept */

/* ---- context ------------------------------------------------------------ */
int mc_ctx_create(int device, mc_ctx **out);
void mc_ctx_destroy(mc_ctx *ctx);
int mc_ctx_set_stream(mc_ctx *ctx, void *hip_stream);   /* NULL = own stream */
void *mc_ctx_get_stream(mc_ctx *ctx);
int mc_ctx_synchronize(mc_ctx *ctx);
const char *mc_ctx_last_error(mc_ctx *ctx);
/* live per-kernel timing with HIP events on the context stream (bench/profiling) */
int mc_ctx_set_timing(mc_ctx *ctx, int enable);
int mc_ctx_set_timing_filter(mc_ctx *ctx, const char *kernel);  /* NULL/"" = every kernel group */
int mc_ctx_get_kernel_time(mc_ctx *ctx, const char *kernel, double *total_ms, int64_t *launches);
int mc_ctx_reset_kernel_times(mc_ctx *ctx);
/* HBM the back-projection's per-batch arrays may take (bytes; 0 = the default: 40 % of the device
   or 65 % of the free memory, whichever is less).  Batches are sized from it (~224 B per pixel);
   a caller sharing the device with its own allocator (or other contexts) keeps the rest. */
int mc_ctx_set_memory_budget(mc_ctx *ctx, int64_t bytes);
/* diagnostics: out[0] = 1 if the library was built with in-kernel invariant checks
   (-DMC_DBG_CHECK=1), out[1 + k] = failures of check kind k so far; n <= 9 */
int mc_debug_counters(mc_ctx *ctx, int64_t *out, int32_t n, int reset);

/* ---- scene input (the S1 output: per-frame mask point sets) ---------------
 * mask_col/label/off are host arrays of length M_in, M_in, M_in+1.
 * mask_pts (length mask_off[M_in]) is a host pointer, or a device pointer
 * when pts_on_device != 0.  Point ids in [0, P); each mask's ids unique;
 * labels in [1, 65535] and unique within a frame; mask_col non-decreasing.  */
int mc_scene_set_masks(mc_ctx *ctx, int64_t num_points, int32_t num_frames, int32_t num_masks_in,
                       const int32_t *mask_col, const int32_t *mask_label, const int64_t *mask_off,
                       const int32_t *mask_pts, int pts_on_device);

/* ---- S1: per-frame mask back-projection ---------------------------------
 * utils/mask_backprojection.py:70-151 (turn_mask_to_point) for a batch of
 * frames: build_point_in_mask_matrix's per-frame loop (construction.py:46-49)
 * without the host round trips.  Scene points: float32 [P,3] (the reference
 * casts to float32 at construction.py:37).  depth float32 [F,H,W] metres,
 * seg uint8 [F,H,W] aligned with depth, intrinsics [F,4] = fx, fy, cx, cy,
 * poses [F,16] row-major camera-to-world; host pointers, or device pointers
 * when on_device != 0.  A frame with an inf pose yields no masks (:73-74); a
 * depth pixel equal to depth_trunc in a frame with mask ids fails the call
 * with MC_ERR_INVALID (the reference raises IndexError at :100).          */
void mc_bp_params_default(mc_bp_params *p);
int mc_scene_set_points(mc_ctx *ctx, int64_t num_points, const float *xyz, int on_device);
int mc_backproject(mc_ctx *ctx, int32_t num_frames, int32_t height, int32_t width, const float *depth,
                   const uint8_t *seg, const double *intrinsics, const double *poses, int on_device,
                   const mc_bp_params *params);
/* the same, with one host pointer per frame (depth_frames[f]: float32 [H,W], seg_frames[f]: uint8
 * [H,W]) as a dataset hands them out (dataset/scannet.py:48-64, construction.py:47-48): the frames
 * are staged through pinned memory by host threads while the previous chunk's DMA runs, with no
 * [F,H,W] host copy.  intrinsics / poses as above (host).                                        */
int mc_backproject_frames(mc_ctx *ctx, int32_t num_frames, int32_t height, int32_t width,
                          const float *const *depth_frames, const uint8_t *const *seg_frames,
                          const double *intrinsics, const double *poses, const mc_bp_params *params);
/* the same from the depth PNGs' raw values (depth_frames[f]: uint16 [H,W]; dataset/scannet.py:51-53,
 * scannetpp.py:168-170, matterport.py:91-93): staged as 2 bytes per pixel instead of 4 and decoded on
 * the device to float32(uint16 / depth_scale) computed in float64 -- the array get_depth returns.  */
int mc_backproject_frames_raw(mc_ctx *ctx, int32_t num_frames, int32_t height, int32_t width,
                              const uint16_t *const *depth_frames, double depth_scale,
                              const uint8_t *const *seg_frames, const double *intrinsics, const double *poses,
                              const mc_bp_params *params);
int mc_backproject_get_info(mc_ctx *ctx, mc_bp_info *info);
/* S1's batching (no reference counterpart; the library's HBM budget, mc_ctx_set_memory_budget):
 * out4 = {frames per batch at the end of the last call, mask-pixel capacity of the per-batch
 * arrays, bytes those arrays hold, batches redone after a mask-pixel overflow (all calls)}       */
int mc_backproject_get_batching(mc_ctx *ctx, int64_t *out4);
/* kept masks in frame order then id order: mask_col (frame index), mask_label
 * (id), mask_off [M+1], mask_pts = sorted unique scene ids (mask_info[id], :148) */
int mc_backproject_get_masks(mc_ctx *ctx, int32_t *mask_col, int32_t *mask_label, int64_t *mask_off,
                             int32_t *mask_pts);
int mc_backproject_get_candidates(mc_ctx *ctx, int32_t *stats /* num_candidates * MC_BP_NSTAT */);
/* mask_pts into a device buffer (stream-ordered on the context stream, no host copy): the
 * frame-sharded path all-gathers the per-rank point lists over RCCL;
 * mask_col / mask_label / mask_off come from mc_backproject_get_masks with mask_pts = NULL */
int mc_backproject_copy_points_device(mc_ctx *ctx, int32_t *mask_pts_dev);

/* the back-projected masks become the graph input (as mc_scene_set_masks, device-resident) */
int mc_scene_use_backprojection(mc_ctx *ctx);

/* ---- S2-S5: graph construction ------------------------------------------ */
int mc_graph_build(mc_ctx *ctx, const mc_graph_params *params);
int mc_graph_get_info(mc_ctx *ctx, mc_graph_info *info);
int mc_graph_get_global_masks(mc_ctx *ctx, int32_t *input_index /* M */);
int mc_graph_get_boundary(mc_ctx *ctx, uint8_t *flags /* P */);
int mc_graph_get_point_in_mask(mc_ctx *ctx, uint16_t *pim /* P*F, row-major */);
int mc_graph_get_point_frame_bits(mc_ctx *ctx, uint64_t *bits /* P*ceil(F/64) */);
int mc_graph_get_visible_frame_bits(mc_ctx *ctx, uint64_t *bits /* M*ceil(F/64) */);
int mc_graph_get_contained(mc_ctx *ctx, int64_t *row_off /* M+1 */, int32_t *col_idx /* nnz */);
int mc_graph_get_undersegment(mc_ctx *ctx, int32_t *ids /* |U| */);
int mc_graph_get_nodes0(mc_ctx *ctx, int32_t *mask_index /* N0 */);
int mc_graph_get_observer_hist(mc_ctx *ctx, uint64_t *hist /* F+1 */);
int mc_graph_get_thresholds(mc_ctx *ctx, float *thr /* 20 */, int32_t *is_int /* 20 */, int32_t *n);

/* get_observer_num_thresholds (construction.py:80-96) on an arbitrary
 * visible-frame matrix: rows of ceil(F/64) little-endian uint64 words.       */
int mc_observer_thresholds(mc_ctx *ctx, int32_t num_rows, int32_t num_frames, const uint64_t *vf_bits,
                           float *thr /* 20 */, int32_t *is_int /* 20 */, int32_t *n);

/* ---- S6 on arbitrary nodes (iterative_clustering on user Node lists) ------
 * Replaces the level-0 nodes: per node the visible-frame bits, the contained
 * mask ids (CSR, unique per row) and the point ids (CSR, unique per row).    */
int mc_nodes_set(mc_ctx *ctx, int32_t num_nodes, int32_t num_frames, int32_t num_masks,
                 int64_t num_points, const uint64_t *vf_bits, const int64_t *c_off,
                 const int32_t *c_idx, const int64_t *pt_off, const int32_t *pt_idx);

/* ---- S6: iterative view-consensus clustering ---------------------------
 * thresholds: host array of n values (np.float32 or the int 1), or NULL to
 * use the thresholds computed on the device by mc_graph_build (no host sync).
 * connect_threshold: args.view_consensus_threshold (compared in float32).   */
int mc_cluster_run(mc_ctx *ctx, const float *thresholds, int32_t n, double connect_threshold);
int mc_cluster_get_info(mc_ctx *ctx, mc_cluster_info *info);
/* Edge capture for the set-order replay: with capacity > 0 the next
 * mc_cluster_run records every edge of every iteration as key = t << 48 | a << 24 | b (a < b,
 * any order); mc_cluster_get_edges gives their count (keys NULL) and the keys
 * (MC_ERR_UNSUPPORTED when more than capacity were found).  Single-process runs only. */
int mc_cluster_set_edge_capture(mc_ctx *ctx, int64_t capacity);
int mc_cluster_get_edges(mc_ctx *ctx, uint64_t *keys, int64_t *n);
int mc_cluster_get_level_sizes(mc_ctx *ctx, int32_t *sizes /* num_iterations+1 */);
/* contained-pool slots of every level (sum of the members' row lengths: the merge's row
 * upper bounds), level 0 = nnz of the initial rows; used for the S6 byte models of bench.py */
int mc_cluster_get_level_caps(mc_ctx *ctx, int32_t *caps /* num_iterations+1 */);
int mc_cluster_get_partition(mc_ctx *ctx, int32_t iteration, int32_t *labels /* N_iteration */);
int mc_cluster_get_edge_counts(mc_ctx *ctx, int64_t *edges /* num_iterations */);
int mc_cluster_get_final_labels(mc_ctx *ctx, int32_t *labels /* N0: object of each level-0 node */);
int mc_cluster_get_objects(mc_ctx *ctx, uint64_t *vf_bits /* K*ceil(F/64) */,
                           int64_t *c_off /* K+1 */, int32_t *c_idx,
                           int64_t *pt_off /* K+1 */, int32_t *pt_idx,
                           int64_t *mask_off /* K+1 */, int32_t *mask_idx /* level-0 node ids */);

/* ---- row-block sharding over processes ------------------------------------
 * One process per GPU, each with its own context holding the same scene (mc_scene_set_masks).
 * After mc_shard_set(ctx, rank, world > 1):
 *   - mc_graph_build runs S2 and S3 (graph/construction.py:98-170) on this rank's block of mask
 *     rows only and leaves MC_SHARD_S3 pending;
 *   - mc_shard_import(MC_SHARD_S3) takes every rank's block, runs the under-segmentation undo,
 *     S5 and this rank's tiles of the S4 observer histogram (:80-96), leaves MC_SHARD_HIST pending;
 *   - mc_shard_import(MC_SHARD_HIST) takes the histogram SUMMED over the ranks and computes the
 *     thresholds (the graph is then complete and identical on every rank);
 *   - mc_cluster_run evaluates the first iteration's N0 x N0 pairs (iterative_clustering.py:20-29)
 *     on the rows a = rank (mod world) and leaves MC_SHARD_FOREST pending;
 *   - mc_shard_import(MC_SHARD_FOREST) unites every rank's union-find forest and runs the rest
 *     of S6 (identical on every rank).
 * The host moves the blocks with its own collectives between the calls: mc_shard_export gives
 * this rank's block (size query with dst_dev = NULL; a stream-ordered copy into a device
 * buffer); all-gather the S3 and FOREST blocks into [world][stride_bytes] in rank order; all-reduce
 * (sum, 64-bit) the HIST block.  mc_shard_pending reports the phase waiting (0 = none).
 * world = 1 restores the single-process path. */
#define MC_SHARD_S3 1
#define MC_SHARD_HIST 2
#define MC_SHARD_FOREST 3
int mc_shard_set(mc_ctx *ctx, int32_t rank, int32_t world);
int mc_shard_pending(mc_ctx *ctx, int32_t *phase);
int mc_shard_export(mc_ctx *ctx, int32_t phase, void *dst_dev, int64_t *bytes);
int mc_shard_import(mc_ctx *ctx, int32_t phase, const void *src_dev, int64_t stride_bytes);

/* ---- native collectives ---------------------------------------------------
 * With an RCCL communicator attached, rank and world come from it and the sharded mc_graph_build /
 * mc_cluster_run run their exchanges themselves, stream-ordered on the context stream (S3 rows and
 * union-find forests: ncclAllGather; the observer histogram: ncclAllReduce sum int64; one max
 * all-reduce + host read for the S3 block stride): nothing is left pending for the host.  This is
 * what the Python collectives in maskclustering_amd/graph_shard.py do through torch.distributed.
 * RCCL is loaded (dlopen librccl.so.1) on first use; MC_ERR_UNSUPPORTED if it is absent.
 *   mc_comm_unique_id   ncclGetUniqueId, on one rank; the caller broadcasts the 128 bytes
 *   mc_ctx_comm_init    ncclCommInitRank on the context's device; the context owns the communicator
 *   mc_ctx_attach_comm  a caller-owned ncclComm_t (NULL detaches: back to the single-process path)
 * A communicator of one rank runs the same exchange flow (each collective an identity). */
#define MC_COMM_ID_BYTES 128
int mc_comm_unique_id(uint8_t id[MC_COMM_ID_BYTES]);
int mc_ctx_comm_init(mc_ctx *ctx, const uint8_t id[MC_COMM_ID_BYTES], int32_t rank, int32_t world);
int mc_ctx_attach_comm(mc_ctx *ctx, void *nccl_comm);

/* ---- post-processing of the clustered objects ----------------------
 * Replaces the compute of utils/post_process.py:173-194 (post_process up to export):
 * dbscan_process (:104-123), filter_point (:40-101), merge_overlapping_objects (:7-37).
 * Inputs are host arrays.  Nodes are the ones post_process keeps (>= 2 masks, :182), their
 * points in list(node.point_ids) order (graph/node.py:45); node masks are indices into the
 * mask table (mask_point_clouds entries) in node.mask_list order, with the frame column of
 * each.  A node mask whose frame is not among the node's visible frames fails with
 * MC_ERR_INVALID (the reference raises IndexError at :69). */
typedef struct mc_pp_params {
    double dbscan_eps;              /* 0.1   post_process.py:104                    */
    int32_t dbscan_min_points;      /* 4     post_process.py:109                    */
    double point_filter_threshold;  /* args.point_filter_threshold, :95             */
    double overlapping_ratio;       /* 0.8   :194                                   */
} mc_pp_params;

typedef struct mc_pp_info {
    int32_t num_objects;   /* DBSCAN objects of all nodes, node order then class order */
    int32_t num_filtered;  /* objects kept by filter_point                            */
    int32_t num_final;     /* objects left after merge_overlapping_objects            */
    int64_t num_entries;   /* node points in total                                    */
    int64_t num_node_masks;
} mc_pp_info;

int mc_pp_run(mc_ctx *ctx, const mc_pp_params *params, int64_t num_points, int32_t num_frames,
              const double *scene_xyz /* P*3 */, const uint64_t *pfm_bits /* P*ceil(F/64) */,
              int32_t num_masks, const int64_t *mask_off /* num_masks+1 */, const int32_t *mask_pts,
              int32_t num_nodes, const uint64_t *node_vf_bits /* num_nodes*ceil(F/64) */,
              const int64_t *node_pt_off /* num_nodes+1 */, const int32_t *node_pts,
              const int64_t *node_mask_off /* num_nodes+1 */, const int32_t *node_masks,
              const int32_t *node_mask_col);
int mc_pp_get_info(mc_ctx *ctx, mc_pp_info *info);
/* entry_object: object of each node point when the point passes the detection-ratio filter
 * and its object is final, else -1; mask_object / mask_coverage: the object each node mask
 * is assigned to (-1: it intersects none) and its coverage;
 * object_state: 0 dropped by filter_point, 1 merged away, 2 final; object_node; bbox
 * (min xyz, max xyz) per DBSCAN object.  Object ids are DBSCAN object ids. */
int mc_pp_get_results(mc_ctx *ctx, int32_t *entry_object, int32_t *mask_object, double *mask_coverage,
                      uint8_t *object_state, int32_t *object_node, double *object_bbox);

/* ---- instance-evaluation match counts -------------------------------
 * Replaces the device part of evaluation/evaluate.py:254-329 (assign_instances_for_scan): per
 * predicted mask k (column k of the [P, K] pred_masks matrix of the prediction npz, non-zero =
 * in the mask, :289): pred_verts[k] = np.count_nonzero (:290), void_intersection[k] (:303) and
 * intersection[k * num_gt + g] = |pred_k ∩ gt instance g| (:308).  gt_instance[p] = index of
 * the ground-truth instance holding point p, or -1. */
int mc_eval_match_counts(mc_ctx *ctx, int64_t num_points, int32_t num_pred, const uint8_t *pred_masks /* P*K */,
                         const int32_t *gt_instance /* P */, int32_t num_gt, const uint8_t *void_flags /* P */,
                         int64_t *pred_verts /* K */, int64_t *void_intersection /* K */,
                         int64_t *intersection /* K*num_gt */);

/* ---- frame decode -------------------------------------------------------
 * Replaces the per-frame host work of dataset/scannet.py:49-54 (get_depth: uint16 / depth_scale
 * as float64, stored float32; matterport.py:92 and scannetpp.py:169 alike) and :68-73
 * (get_segmentation(align_with_depth=True): cv2.resize(seg, (W, H), INTER_NEAREST)) for a batch of
 * frames.  Inputs are host arrays, or device pointers when inputs_on_device; outputs are device
 * pointers (e.g. the depth / seg arrays mc_backproject reads).  depth or seg may be NULL. */
int mc_frames_decode(mc_ctx *ctx, int32_t num_frames, int32_t height, int32_t width,
                     const uint16_t *depth /* F*H*W */, double depth_scale, int32_t seg_height, int32_t seg_width,
                     const uint8_t *seg /* F*seg_height*seg_width */, int inputs_on_device,
                     float *depth_out /* device, F*H*W */, uint8_t *seg_out /* device, F*H*W */);

/* ---- open-vocabulary label query ---------------------------------------
 * Replaces the per-object compute of semantics/open-voc_query.py:32-53: for object k, the mean of
 * its representative masks' features (rows obj_rows[obj_off[k] .. obj_off[k+1]) of the
 * num_rows x dim float32 table, summed in that order), its similarity with every label text
 * feature (num_labels x dim), exp(temperature * sim), the softmax and its first argmax (NaN
 * first, like np.argmax; -1 for an object without representative masks).  Float32 like the
 * reference except the dot products, which are summed in float64 and rounded once (the
 * reference's BLAS order is its own). */
int mc_openvoc_query(mc_ctx *ctx, int32_t num_objects, const int64_t *obj_off, const int32_t *obj_rows,
                     int32_t num_rows, int32_t dim, const float *features, int32_t num_labels,
                     const float *label_features, float temperature, int32_t *out_label);

/* host utility: packed little-endian bit rows (bit c of word c/64 = column c) -> one byte per
 * column, rows * ncols bytes (the dense bool point_frame_matrix the reference's callers read,
 * graph/construction.py:40,52), split over host threads.                                      */
int mc_bits_unpack(const uint64_t *words, int64_t rows, int32_t words_per_row, int32_t ncols, uint8_t *out);

/* host utility: the reference's container ORDERS of the clustering result (graph/iterative_clustering.py:5-10
 * + graph/node.py:24-37 under networkx 3.x's _plain_bfs and CPython's set tables; mc_setorder.inl).
 * Iterations t = 0 .. num_levels-1 with level_sizes[t] nodes; iteration t's edges (a, b), a != b, are
 * edge_a/edge_b[edge_off[t] .. edge_off[t+1]) (level_sizes[t+1] must be the number of components of t).
 * Level-0 node i's point set was made by adding pts[pt_off[i] .. pt_off[i+1]) in order to an empty set.
 * Out (caller-allocated, K = *num_objects = components of the last iteration <= level_sizes[T-1]):
 *   obj_mask_off [K+1] + mask_order [level_sizes[0]]: final node k's mask_list as level-0 node indices;
 *   obj_pt_off [K+1] + obj_pts [<= pt_off[level_sizes[0]]]: list(final node k's point_ids);
 *   son_off [K+1] + son_order [level_sizes[T-1]]: the last iteration's members of k in set order;
 *   labels [sum_t level_sizes[t]] (NULL: not returned): component of every node of every iteration.
 * num_threads <= 0: all host threads.                                                                 */
int mc_setorder_replay(int32_t num_levels, const int32_t *level_sizes, const int64_t *edge_off,
                       const int32_t *edge_a, const int32_t *edge_b, const int64_t *pt_off, const int32_t *pts,
                       int32_t num_threads, int32_t *num_objects, int64_t *obj_mask_off, int32_t *mask_order,
                       int64_t *obj_pt_off, int32_t *obj_pts, int64_t *son_off, int32_t *son_order,
                       int32_t *labels);

/* The same in two calls, so that the level-0 sets are built while the device clusters: begin takes
 * level-0 node i's points as pts[node_start[i] .. node_start[i] + node_len[i]) (rows of the caller's
 * mask CSR, no flattened copy) and, with async_build != 0, builds the sets on a background thread
 * (the caller keeps node_start / node_len / pts alive until finish or free); finish waits for it and
 * replays the iterations exactly as mc_setorder_replay (outputs as there; obj_pts holds at most
 * sum(node_len)).  finish is called at most once; free joins and releases (also after an error). */
typedef struct mc_setorder mc_setorder;
int mc_setorder_begin(int32_t num_nodes, const int64_t *node_start, const int64_t *node_len, const int32_t *pts,
                      int32_t num_threads, int async_build, mc_setorder **out);
int mc_setorder_finish(mc_setorder *h, int32_t num_levels, const int32_t *level_sizes, const int64_t *edge_off,
                       const int32_t *edge_a, const int32_t *edge_b, int32_t *num_objects, int64_t *obj_mask_off,
                       int32_t *mask_order, int64_t *obj_pt_off, int32_t *obj_pts, int64_t *son_off,
                       int32_t *son_order, int32_t *labels);
void mc_setorder_free(mc_setorder *h);

#ifdef __cplusplus
}
#endif
#endif /* MCGRAPH_H */
