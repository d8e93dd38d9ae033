/*
 * ofx.h — C ABI of the MI355X-native non-rigid TSDF fusion hot path (libofx.so).
 *
 * Drop-in boundary for remmel/OcclusionFusion's fusion core. Every entry point
 * takes plain device pointers + sizes and a HIP stream; no torch / numpy types
 * cross this ABI. All work is stream-ordered and asynchronous unless an entry
 * point says otherwise. Caller owns every buffer; the library owns only scratch
 * tied to an opaque handle (GN solver). Errors: int status (0 ok, <0 error) and
 * ofx_last_error() (thread-local string). Nothing throws across the ABI.
 *
 * Reference interfaces replaced (file:line in /root/reference):
 *   ofx_volume_reset        TSDFVolume.__init__ dense init tsdf=1, w=0, c=0   fusion_with_occlusion/tsdf.py:133-141
 *   ofx_volume_to_dense     TSDFVolume.get_volume (D2H on request)          tsdf.py:673-680
 *   ofx_volume_from_dense   TSDFVolume.load_volume                          tsdf.py:689-702
 *   ofx_pack_color          TSDFVolume.update colour folding                tsdf.py:545-566
 *   ofx_skin_volume_bricks  WarpField.skin_tsdf (cache build, brick cull)   warpfield.py:131-141
 *   ofx_skin_volume         WarpField.skin over TSDFVolume.world_pts       warpfield.py:83-129, tsdf.py:294-307
 *   ofx_skin_palette        (layout only) per-brick node palette of the skin_tsdf cache, warpfield.py:131-141
 *   ofx_skin_points         WarpField.skin(points, nodes)                  warpfield.py:83-129
 *                           (k-NN twin of csrc compute_pixel_anchors_euclidean, csrc/cpu/graph_proc.cpp:610-709)
 *   ofx_pack_nodes          Registration.deform_ED gathers of R, t, g       NonRigidICP/model/registration_fusion.py:168-170
 *   ofx_integrate           WarpField.deform_tsdf + TSDFVolume.integrate    warpfield.py:369-380, tsdf.py:378-494
 *                           (fused: skin cache -> ED warp -> project -> SDF/weight/colour update)
 *   ofx_integrate_palette   same, node records staged per brick in LDS      warpfield.py:369-380, tsdf.py:442-494
 *   ofx_integrate_palette_cull  same, bricks that provably update nothing skipped (per-frame cull)
 *   ofx_integrate_points    TSDFVolume.integrate of given (deformed) points  tsdf.py:442-494
 *   ofx_raycast             (new) depth / normal / colour images of the TSDF  — (no reference twin)
 *   ofx_deform_points       ED_warp / deform_ED / deform_mesh / normals     NonRigidICP/model/geometry.py:9-25,
 *                                                                          registration_fusion.py:157-184, warpfield.py:312-367
 *   ofx_deform_points_lbs   WarpField.deform_lbs / deform_lbs_cuda (origin form) warpfield.py:208-266,270-305
 *   ofx_visibility          TSDFVolume.check_visibility                     tsdf.py:576-612
 *   ofx_truncated_region    TSDFVolume.compute_truncated_region            tsdf.py:704-745
 *   ofx_mesh_*              measure.marching_cubes in get_mesh / get_point_cloud, colours tsdf.py:748-809
 *   ofx_backproject_depth   image_proc.backproject_depth (csrc float/ushort) utils/image_proc.py:335-349,
 *                                                                          csrc/cpu/image_proc.cpp:351-401
 *   ofx_depth_mesh_*        compute_mesh_from_depth (pixel-grid mesh)       csrc/cpu/image_proc.cpp:405-545
 *                           (EDGraph.create_mesh_from_depth, WarpField.skin of an image: embedded_deformation_graph.py:95-151,
 *                           warpfield.py:160-175)
 *   ofx_depth_to_pc         Registration.optimize target cloud: depth_2_pc, NonRigidICP/model/geometry.py:44-59,
 *                           mask compaction, map_pixel_to_pcd              registration_fusion.py:104-109,388-395
 *   ofx_pixel_anchors_euclidean  csrc compute_pixel_anchors_euclidean     csrc/cpu/graph_proc.cpp:610-709
 *   ofx_pixel_anchors_geodesic   csrc compute_pixel_anchors_geodesic      csrc/cpu/graph_proc.cpp:483-608
 *   ofx_remap_anchors       csrc update_pixel_anchors                       csrc/cpu/graph_proc.cpp:934-961
 *   ofx_knn_points          KDTree.query (pykdtree) in WarpField.find_unreachable_nodes  warpfield.py:462-485
 *   ofx_graph_create/destroy/adjacency  mesh vertex adjacency (std::set per vertex)  csrc/cpu/graph_proc.cpp:174-186
 *   ofx_erode_mesh          csrc erode_mesh                                 csrc/cpu/graph_proc.cpp:17-77
 *   ofx_sample_nodes        csrc sample_nodes (randomShuffle = false)       csrc/cpu/graph_proc.cpp:79-136
 *   ofx_edges_geodesic      csrc compute_edges_geodesic                     csrc/cpu/graph_proc.cpp:155-300
 *   ofx_edges_euclidean     csrc compute_edges_euclidean                    csrc/cpu/graph_proc.cpp:302-356
 *   ofx_node_edge_cleanup   csrc node_and_edge_clean_up                     csrc/cpu/graph_proc.cpp:388-438
 *   ofx_compute_clusters    csrc compute_clusters                           csrc/cpu/graph_proc.cpp:440-481
 *                           (callers: EDGraph, fusion_with_occlusion/embedded_deformation_graph.py:153-380,496-609)
 *   ofx_reduce_graph        EDGraph.get_reduced_graph                       embedded_deformation_graph.py:382-477
 *   ofx_graph_downsample    EDGraph.create_graph_pyramid down-sampling      embedded_deformation_graph.py:278-299
 *   ofx_gn_*                DeformNet.optimize Gauss-Newton (JᵀJ, Jᵀr, LU)   model/model.py:222-859 (+ LinearSolverLU :59-86)
 *                           DeformNet.arap (params.mode = OFX_GN_ARAP)       model/model.py:1639-1986
 *                           (LU replaced by warm-started block-Jacobi PCG; ofx_gn_stats: per-step diagnostics)
 */
#ifndef OFX_H
#define OFX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OFX_ABI_VERSION 5

typedef void* ofx_stream_t; /* hipStream_t; NULL = legacy default stream */

enum {
  OFX_OK = 0,
  OFX_ERR_ARG = -1,      /* bad argument / shape */
  OFX_ERR_HIP = -2,      /* HIP runtime error */
  OFX_ERR_RANGE = -3,    /* size limit exceeded (e.g. > 65534 nodes) */
  OFX_ERR_STATE = -4,    /* call order violated */
  OFX_ERR_ALLOC = -5
};

const char* ofx_last_error(void);
int ofx_abi_version(void);

/* Voxel volume: dense grid (reference C-order semantics), stored on device as
 * 8x8x8 bricks, brick-major. A shard owns bricks [brick_x0, brick_x1) along x. */
typedef struct ofx_volume_desc {
  int32_t dim[3];       /* Dx, Dy, Dz (TSDFVolume._vol_dim) */
  int32_t brick_x0;     /* first brick column along x owned by this shard */
  int32_t brick_x1;     /* one past the last (full volume: ceil(Dx/8)) */
  int32_t semantics;    /* integrate arithmetic: OFX_SEM_CPU (0) or OFX_SEM_PYCUDA (1) */
  float origin[3];      /* TSDFVolume._vol_origin (f32) */
  float _pad1;
  double voxel_size;    /* TSDFVolume._voxel_size (f64) */
  double trunc_margin;  /* TSDFVolume._trunc_margin (0.04) */
} ofx_volume_desc;

/* Integrate semantics (ofx_volume_desc.semantics). The reference has two integrate paths that compute
 * different numbers:
 *   OFX_SEM_CPU    numba/numpy CPU branch, tsdf.py:442-494: f64 projection, round-half-even pixels,
 *                  update iff depth > 0 and d - z >= -trunc, plain d - z.
 *   OFX_SEM_PYCUDA pycuda kernel, tsdf.py:192-288 (used when fopt.gpu and pycuda import): f32 throughout,
 *                  pixel = (int)roundf(f32(f·x/z + c) + 0.5) (half away from zero), skip iff depth == 0,
 *                  (d - z) scaled by the ray factor sqrt(1 + mx² + my²) of the integer pixel, roundf colours. */
enum { OFX_SEM_CPU = 0, OFX_SEM_PYCUDA = 1 };

typedef struct ofx_camera {
  float fx, fy, cx, cy; /* cam_intr (cast to f32 as tsdf.py:357) */
  int32_t width, height;
} ofx_camera;

/* number of voxel slots (bricks*512) a shard stores */
int ofx_volume_num_slots(const ofx_volume_desc* desc, int64_t* n_slots);

int ofx_volume_reset(const ofx_volume_desc* desc, float* tsdf, float* weight, float* color, ofx_stream_t s);
/* bricked shard -> C-order dense (Dx_shard, Dy, Dz) where Dx_shard = min(8*x1,Dx) - 8*x0 */
int ofx_volume_to_dense(const ofx_volume_desc* desc, const float* bricked, float* dense, ofx_stream_t s);
int ofx_volume_from_dense(const ofx_volume_desc* desc, const float* dense, float* bricked, ofx_stream_t s);

/* rgb (3,H,W) f32 in [0,1] -> packed colour (H,W) f32 (tsdf.py:561-562) */
int ofx_pack_color(const float* rgb, int32_t height, int32_t width, float* packed, ofx_stream_t s);

/* Skinning of the voxel grid.
 * Step 1: list the shard's bricks that can hold a skin-valid voxel (>= K nodes within
 *         4*node_coverage of the brick). brick_list: int32[num_bricks], count: device int32[1].
 * Step 2: per-voxel k-NN for the listed bricks -> anchors uint16[n_list*512*4] (0xFFFF = -1),
 *         weights f32[n_list*512*4]; slot = list position.                                */
int ofx_skin_volume_bricks(const ofx_volume_desc* desc, const float* nodes, int32_t n_nodes,
                           double node_coverage, int32_t k, int32_t* brick_list, int32_t* count,
                           ofx_stream_t s);
int ofx_skin_volume(const ofx_volume_desc* desc, const float* nodes, int32_t n_nodes, double node_coverage,
                    int32_t k, const int32_t* brick_list, int32_t n_list, uint16_t* anchors, float* weights,
                    ofx_stream_t s);
/* Node palette of the bricked skin cache (MI355X-specific, no reference twin): per listed brick the
 * ascending distinct anchors of its skin-valid voxels, pal_ids u16[n_list*OFX_PALETTE], count
 * pal_n i32[n_list] (> OFX_PALETTE: overflow, palette unused), and per voxel the anchors as palette
 * ranks local_anchors u8[n_list*512*4] (0xFF: skin-invalid voxel / unused slot). */
#define OFX_PALETTE 64
int ofx_skin_palette(const uint16_t* anchors, int32_t n_list, int32_t k, int32_t n_nodes, uint16_t* pal_ids,
                     int32_t* pal_n, uint8_t* local_anchors, ofx_stream_t s);
/* Skinning of arbitrary points: anchors int32[P*K] (-1 beyond 4σ), weights f32[P*K], valid u8[P] */
int ofx_skin_points(const float* points, int64_t n_points, const float* nodes, int32_t n_nodes,
                    double node_coverage, int32_t k, int32_t* anchors, float* weights, uint8_t* valid,
                    ofx_stream_t s);
/* Expand the bricked skin cache to C-order (V,4) int32 / f32 / valid u8 (testing & API parity). */
int ofx_skin_volume_to_dense(const ofx_volume_desc* desc, const int32_t* brick_list, int32_t n_list,
                             const uint16_t* anchors, const float* weights, int32_t k, int32_t* anchors_out,
                             float* weights_out, uint8_t* valid_out, ofx_stream_t s);

/* Node transforms (node-relative, as Registration.deform_ED uses them):
 * R f32[N*9] row-major, T f32[N*3], g f32[N*3] -> packed f32[N*16], 64-B records interleaved for
 * packed-f32 warps: [R00 R10 R01 R11 | R02 R12 g0 g1 | t0 t1 R20 R21 | R22 g2 t2 0] */
int ofx_pack_nodes(const float* R, const float* T, const float* g, int32_t n_nodes, float* packed,
                   ofx_stream_t s);

/* Fused warp + integrate of one frame into the shard.
 *   warp = 0 : source frame — every voxel, world position, no skin (tsdf.py:395-398); with brick_list
 *              non-NULL (CPU semantics only) just the n_list listed bricks (a hash-bucket shard's own)
 *   warp = 1 : bricks in brick_list, ED-warped positions, skin-valid voxels only (tsdf.py:401,464)
 * color_im / color may be NULL (no colour integration). n_updated (device u32, one entry per launched
 * brick: n_list when a list is given, all shard bricks otherwise) receives per-brick update counts, may
 * be NULL. */
int ofx_integrate(const ofx_volume_desc* desc, const ofx_camera* cam, const float* depth, const float* color_im,
                  int32_t warp, const float* packed_nodes, int32_t n_nodes, int32_t k,
                  const int32_t* brick_list, int32_t n_list, const uint16_t* anchors, const float* weights,
                  double obs_weight, float* tsdf, float* weight, float* color,
                  uint32_t* n_updated, ofx_stream_t s);

/* ofx_integrate (warp = 1) with the skin cache's node palette (ofx_skin_palette): each brick's node
 * records are staged once in LDS. Bit-identical results; bricks with pal_n > OFX_PALETTE fall back
 * to the global anchors. */
int ofx_integrate_palette(const ofx_volume_desc* desc, const ofx_camera* cam, const float* depth,
                          const float* color_im, const float* packed_nodes, int32_t n_nodes, int32_t k,
                          const int32_t* brick_list, int32_t n_list, const uint16_t* anchors, const float* weights,
                          const uint16_t* pal_ids, const int32_t* pal_n, const uint8_t* local_anchors,
                          double obs_weight, float* tsdf, float* weight, float* color, uint32_t* n_updated,
                          ofx_stream_t s);

/* ofx_integrate_palette with a per-frame brick cull in front (CPU semantics, k = 4; otherwise it is
 * ofx_integrate_palette): per 8x8 pixel tile the largest depth (tile_scratch: f32[ceil(W/8)*ceil(H/8)]), then per
 * listed brick a conservative box of its warped voxels (each palette node's rigid image of the brick, scaled by the
 * skin weights' sum range) tested against the camera and those tiles; bricks that provably update no voxel are
 * skipped (active: u8[n_list] receives the flags; n_updated gets 0 for them). Bit-identical results. MI355X-specific:
 * no reference twin (the reference walks every voxel, tsdf.py:442-494). */
int ofx_integrate_palette_cull(const ofx_volume_desc* desc, const ofx_camera* cam, const float* depth,
                               const float* color_im, const float* packed_nodes, int32_t n_nodes, int32_t k,
                               const int32_t* brick_list, int32_t n_list, const uint16_t* anchors, const float* weights,
                               const uint16_t* pal_ids, const int32_t* pal_n, const uint8_t* local_anchors,
                               double obs_weight, float* tsdf, float* weight, float* color, uint32_t* n_updated,
                               float* tile_scratch, uint8_t* active, ofx_stream_t s);

/* Profiling hook (process-wide): returns (and resets) the device time of the warped integrate kernel launches
 * (ofx_integrate warp = 1, ofx_integrate_palette) recorded since the last call, from hipEvents recorded by the
 * library around each launch on its stream (synchronises on them), and their count; `enable` switches
 * recording for the following launches. */
int ofx_integrate_timing(int32_t enable, double* kernel_ms, int64_t* launches);

/* Integrate of explicit (already deformed) points: point p updates the voxel with C-order id voxel_ids[p]
 * (i·Dy·Dz + j·Dz + k) as TSDFVolume.integrate does for pts from WarpField.deform_tsdf (tsdf.py:442-494,
 * warpfield.py:369-380); valid (u8, may be NULL) masks points. Same arithmetic as ofx_integrate (CPU or
 * pycuda semantics). Voxel ids must be distinct; ids outside this shard are ignored. n_updated (one u32,
 * may be NULL) is incremented by the number of updated voxels. */
int ofx_integrate_points(const ofx_volume_desc* desc, const ofx_camera* cam, const float* depth, const float* color_im,
                         const float* points, const int64_t* voxel_ids, const uint8_t* valid, int64_t n_points,
                         double obs_weight, float* tsdf, float* weight, float* color, uint32_t* n_updated,
                         ofx_stream_t s);

/* TSDF raycast (new capability; the reference has none — parity unpinned, restated by the oracle): per pixel
 * of `cam` (identity pose), march the ray from max(z_near, volume entry) to min(z_far, volume exit) through the
 * trilinear tsdf (unobserved voxels and the outside count as +1), coarse steps of 0.8·trunc while the sample
 * is >= 0.999, one-voxel steps otherwise; the first + -> - sign change, linearly refined, is the surface.
 * depth f32[H*W] (z, 0 = miss); normals f32[H*W*3] (normalised central differences, may be NULL); colors
 * f32[H*W] (packed colour of the nearest voxel, may be NULL; color may be NULL then). Needs the whole volume
 * (brick range [0, nbx)). */
int ofx_raycast(const ofx_volume_desc* desc, const ofx_camera* cam, const float* tsdf, const float* weight,
                const float* color, float z_near, float z_far, float* depth, float* normals, float* colors,
                ofx_stream_t s);

/* ED warp of points: out = Σ w (R(x-g)+g+t) for valid points, x otherwise.
 * normals = 1: WarpField.deform_normals semantics (R only, renormalised). valid may be NULL (all valid). */
int ofx_deform_points(const float* points, int64_t n_points, const int32_t* anchors, const float* weights,
                      const uint8_t* valid, int32_t k, const float* packed_nodes, int32_t n_nodes,
                      int32_t normals, float* out, ofx_stream_t s);

/* WarpField.deform_lbs (origin-form LBS, the use_pytorch=False branch of WarpField.deform):
 * out = Σ_{k: w_k != 0} w_k (R_k x + t_k) for valid points, x otherwise; rotations f32[N*9] row-major,
 * translations f32[N*3] in origin form (t = -R g + g + T). Anchors must be in [0, n_nodes) where w != 0. */
int ofx_deform_points_lbs(const float* points, int64_t n_points, const int32_t* anchors, const float* weights,
                          const uint8_t* valid, int32_t k, const float* rotations, const float* translations,
                          int32_t n_nodes, float* out, ofx_stream_t s);

/* check_visibility: valid u8[P], depth_diff f64[P] */
int ofx_visibility(const float* points, int64_t n_points, const ofx_camera* cam, const float* depth,
                   double trunc_margin, uint8_t* valid, double* depth_diff, ofx_stream_t s);
/* The same check with the projection in f32, as numba runs cam2pix on an f32 point array: get_visible_nodes on
 * the f32 deformed nodes (tsdf.py:614-638 -> 599-612 -> 351-364); depth lookup and depth_diff in f64 */
int ofx_visibility_f32(const float* points, int64_t n_points, const ofx_camera* cam, const float* depth,
                       double trunc_margin, uint8_t* valid, double* depth_diff, ofx_stream_t s);

/* ---------------- Surface extraction ----------------
 * Voxel-index coordinates as skimage returns. ofx_truncated_region / ofx_mesh_count take the whole volume;
 * ofx_mesh_count_range takes a shard whose stored bricks include a halo (see there). */
/* TSDFVolume.compute_truncated_region (tsdf.py:704-745): mask u8 per voxel slot (bricked layout) */
int ofx_truncated_region(const ofx_volume_desc* desc, const float* tsdf, double max_diff, uint8_t* mask,
                         ofx_stream_t s);
/* Marching cubes (measure.marching_cubes at tsdf.py:755,794), two phases on an opaque handle:
 * ofx_mesh_count classifies cells and sizes the output (synchronises the stream), the caller allocates,
 * ofx_mesh_emit writes verts f32[V*3] (voxel coordinates), faces i32[F*3] and optionally normals
 * f32[V*3] (unit, towards increasing tsdf), values f32[V], keys i64[V] (= C-index(edge start)*3 + axis).
 * use_mask = 0: every cell (get_point_cloud); use_mask = 1 with mask = NULL: the volume's truncated region
 * with max_diff (get_mesh, tsdf.py:792); with a mask (bricked u8): that mask. A cell [c, c+1]^3 is
 * processed iff the mask holds at its far corner c+1. */
int ofx_mesh_create(void** handle);
int ofx_mesh_destroy(void* handle);
int ofx_mesh_count(void* handle, const ofx_volume_desc* desc, const float* tsdf, const uint8_t* mask, double max_diff,
                   int32_t use_mask, float level, int64_t* n_verts, int64_t* n_faces, ofx_stream_t s);
int ofx_mesh_emit(void* handle, float* verts, int32_t* faces, float* normals, float* values, int64_t* keys,
                  ofx_stream_t s);
/* Sharded marching cubes: like ofx_mesh_count on a shard desc (bricks [brick_x0, brick_x1), holding the
 * shard's own bricks plus halo bricks copied from its neighbours), processing only the cells whose far corner
 * x lies in [px0, px1) — the shard's own planes. px0 >= 8*brick_x0 + 2 unless brick_x0 = 0, px1 <= 8*brick_x1 - 2
 * unless the shard reaches the volume's end (the truncated-region test and the vertex normals read ±2 planes).
 * The emitted vertices are those the shard's cells use, in global order (keys identify them across shards);
 * the full volume's mesh is the key-merge of the shards' meshes (occlusionfusion_amd.sharding). */
int ofx_mesh_count_range(void* handle, const ofx_volume_desc* desc, const float* tsdf, const uint8_t* mask,
                         double max_diff, int32_t use_mask, float level, int32_t px0, int32_t px1, int64_t* n_verts,
                         int64_t* n_faces, ofx_stream_t s);
/* get_mesh / get_point_cloud epilogue (tsdf.py:757-767,796-807): world = verts*f32(voxel_size) + origin
 * (f32, may be NULL) and colours u8[V*3] = [r,g,b] of the voxel nearest each vertex (may be NULL). */
int ofx_mesh_finish(const ofx_volume_desc* desc, const float* color, const float* verts, int64_t n_verts,
                    float* world, uint8_t* colors, ofx_stream_t s);

/* ---------------- Correspondence front-end ---------------- */
/* backproject_depth: point_image f32[3*H*W] (planar x, y, z); pixels with depth <= 0 are left untouched
 * (the reference zero-fills before the call). depth is f32[H*W] metres (is_u16 = 0) or u16[H*W] scaled by
 * 1/normalizer (is_u16 = 1). Arithmetic as the C++: f32 d*(x-cx)/fx, correctly rounded. */
int ofx_backproject_depth(const void* depth, int32_t is_u16, int32_t height, int32_t width, float fx, float fy, float cx,
                          float cy, float normalizer, float* point_image, ofx_stream_t s);
/* compute_mesh_from_depth on a planar point image f32[3*H*W]; handle owns scratch (also used by
 * ofx_depth_to_pc). count sizes the output (synchronises the stream); emit writes vertices f32[V*3],
 * vertex_pixels i32[V*2] (x, y; may be NULL) and faces i32[F*3], numbered exactly as the sequential C++. */
int ofx_depth_mesh_create(void** handle);
int ofx_depth_mesh_destroy(void* handle);
int ofx_depth_mesh_count(void* handle, const float* point_image, int32_t height, int32_t width,
                         float max_triangle_distance, int64_t* n_verts, int64_t* n_faces, ofx_stream_t s);
int ofx_depth_mesh_emit(void* handle, float* vertices, int32_t* vertex_pixels, int32_t* faces, ofx_stream_t s);
/* depth_2_pc(depth, K) (f64 arithmetic, rounded to f32) of the pixels with depth > 0, row-major:
 * points f32[capacity H*W*3], pix_map i64[H*W] (point index or -1; may be NULL), n_points: DEVICE int32.
 * Asynchronous (no host sync). */
int ofx_depth_to_pc(void* handle, const float* depth, int32_t height, int32_t width, double fx, double fy, double cx,
                    double cy, float* points, int64_t* pix_map, int32_t* n_points, ofx_stream_t s);

/* ---------------- Standalone skinning / anchors ---------------- */
/* csrc twins, exact (Eigen summation order, list tie order, f32 weights): outputs (H, W, 4) images,
 * anchors i32 (-1 = none) and weights f32, fully (re)initialised by the call. point_image planar f32[3*H*W]. */
int ofx_pixel_anchors_euclidean(const float* nodes, int32_t n_nodes, const float* point_image, int32_t height,
                                int32_t width, float node_coverage, int32_t* pixel_anchors, float* pixel_weights,
                                ofx_stream_t s);
/* node_to_vertex_distance f32[N*V] (row per node, < 0 = unreachable), valid_nodes_mask i32[N],
 * vertex_pixels i32[V*2] (x, y). */
int ofx_pixel_anchors_geodesic(const float* node_to_vertex_distance, const int32_t* valid_nodes_mask, int32_t n_nodes,
                               int64_t n_vertices, const int32_t* vertex_pixels, int32_t width, int32_t height,
                               float node_coverage, int32_t* pixel_anchors, float* pixel_weights, ofx_stream_t s);
/* anchors[i] = id_map[anchors[i]] for anchors[i] != -1 (in place). An anchor with no mapping (outside
 * [0, n_map) or mapped to -1; std::map::at would throw) is left as is and counted into *n_missing (DEVICE
 * int32, accumulated: zero it first). */
int ofx_remap_anchors(int32_t* anchors, int64_t n, const int32_t* id_map, int32_t n_map, int32_t* n_missing,
                      ofx_stream_t s);
/* k nearest nodes (k <= 8) of each point: idx i32[P*k] ascending by (squared distance, node id), -1 past
 * n_nodes; sq_dist f32[P*k] = (dx²+dy²)+dz² in f32. */
int ofx_knn_points(const float* points, int64_t n_points, const float* nodes, int32_t n_nodes, int32_t k, int32_t* idx,
                   float* sq_dist, ofx_stream_t s);

/* ---------------- ED-graph construction ----------------
 * Bit-exact with the compiled reference C++ (tests/test_gpu_graph.py). Graph building runs at init and on
 * graph updates; these entry points synchronise the stream where an output size or a convergence test is
 * needed. A handle keeps the mesh's vertex adjacency; it references (does not copy) vertices f32[V*3] and
 * faces i32[F*3], which must stay alive until ofx_graph_destroy. */
int ofx_graph_create(const float* vertices, int64_t n_vertices, const int32_t* faces, int64_t n_faces, void** handle,
                     ofx_stream_t s);
int ofx_graph_destroy(void* handle);
int ofx_graph_adjacency(void* handle, int32_t* rowptr, int32_t* col, int64_t* n_col, ofx_stream_t s);
/* non_eroded u8[V] */
int ofx_erode_mesh(void* handle, int32_t n_iterations, int32_t min_neighbors, uint8_t* non_eroded, ofx_stream_t s);
/* node_positions f32[V*3] / node_indices i32[V] capacity; *n_nodes written (host); *n_rounds: batches of the
 * single-workgroup greedy form (meshes up to ~1.29M vertices), else launches of the parallel round form
 * (OFX_SN_ROUNDS=1 forces it; OFX_SN_STAMPS=1 prints the greedy form's phase times to stderr) */
int ofx_sample_nodes(void* handle, const uint8_t* non_eroded, float node_coverage, int32_t use_only_non_eroded,
                     float* node_positions, int32_t* node_indices, int64_t* n_nodes, int64_t* n_rounds,
                     ofx_stream_t s);
/* graph_edges i32[N*K] (-1 padded), weights / distances f32[N*K] (0 padded), node_to_vertex_distances f32[N*V]
 * (-1 where unvisited; may be NULL). valid_vertices u8[V] may be NULL (all valid). K <= 16. Reaching an
 * invalid vertex with allow_only_valid_vertices (the reference calls exit(0)) returns OFX_ERR_STATE. */
int ofx_edges_geodesic(void* handle, const uint8_t* valid_vertices, const int32_t* node_indices, int32_t n_nodes,
                       int32_t n_max_neighbors, float node_coverage, int32_t allow_only_valid_vertices,
                       int32_t enforce_total_num_neighbors, int32_t* graph_edges, float* graph_edges_weights,
                       float* graph_edges_distances, float* node_to_vertex_distances, ofx_stream_t s);
/* nodes the last ofx_edges_geodesic on this handle settled with the sequential heap kernel (distance ties
 * the parallel relaxation cannot order, or a neighbourhood larger than its LDS table); the rest were settled
 * by the parallel form. OFX_GEO_SEQ=1 in the environment forces the sequential kernel for every node,
 * OFX_GEO_BIG=1 the 16384-slot parallel form (tests / tuning; results are identical either way). */
int ofx_graph_geodesic_sequential(void* handle, int64_t* n_nodes);
/* one level of EDGraph.create_graph_pyramid's down-sampling (embedded_deformation_graph.py:278-299):
 * down_idx i32[n] (first *n_down valid: kept node indices, ascending), up_idx i32[n] (per node: argmin index
 * INTO the kept list, as the reference). At most 8192 kept nodes (else OFX_ERR_RANGE). Synchronises. */
int ofx_graph_downsample(const float* node_positions, int32_t n_nodes, double node_coverage, int32_t* down_idx,
                         int32_t* up_idx, int32_t* n_down, ofx_stream_t s);
int ofx_edges_euclidean(const float* node_positions, int32_t n_nodes, int32_t n_max_neighbors, int32_t* graph_edges,
                        ofx_stream_t s);
/* valid_in / valid_out u8[N] (may alias) */
int ofx_node_edge_cleanup(const int32_t* graph_edges, int32_t n_nodes, int32_t max_neighbors, const uint8_t* valid_in,
                          uint8_t* valid_out, ofx_stream_t s);
/* clusters i32[N]; cluster_sizes i32[N] capacity (may be NULL); *n_clusters (host) */
int ofx_compute_clusters(const int32_t* graph_edges, int32_t n_nodes, int32_t max_neighbors, int32_t* clusters,
                         int32_t* cluster_sizes, int32_t* n_clusters, ofx_stream_t s);

/* get_reduced_graph: keep the nodes with valid_nodes_mask (u8[N]) in order; edges to removed nodes are
 * dropped (compacted left, ids remapped) and the weights renormalised by f32(f64(np.sum) + 1e-6) as numpy 1.26
 * evaluates it; if no node is removed the rows are copied unchanged. clusters / clusters_out may be NULL.
 * Outputs sized for N rows; *n_kept (host). */
int ofx_reduce_graph(const uint8_t* valid_nodes_mask, int32_t n_nodes, int32_t max_neighbors, const float* nodes,
                     const int32_t* edges, const float* edges_weights, const float* edges_distances,
                     const int32_t* clusters, float* nodes_out, int32_t* edges_out, float* weights_out,
                     float* distances_out, int32_t* clusters_out, int32_t* n_kept, ofx_stream_t s);

/* ---------------- Gauss-Newton (DeformNet.optimize) ---------------- */
typedef struct ofx_gn_params {
  int32_t num_iter;          /* 10 (model.py:91) */
  int32_t use_edge_weighting;/* 0 (custom_settings.py:41) */
  int32_t pcg_max_iter;      /* inner PCG cap */
  int32_t pcg_warm;          /* 1: start each GN step's PCG from the Galerkin projection of b onto the
                                last 4 GN-step solutions (A-norm optimal in that span); 0: x0 = 0 */
  double lambda_flow;        /* 0   (model.py:96) — squared weights, sqrt taken inside (model.py:374-377) */
  double lambda_depth;       /* 1   (model.py:101) */
  double lambda_arap;        /* 0.5 (model.py:105) */
  double lambda_motion;      /* 1   (model.py:108) */
  double lm_factor;          /* 1e-7 (model.py:111) */
  double stop_loss_diff;     /* 1   (model.py:114) */
  double pcg_tol;            /* relative residual target of the inner solve */
  int32_t mode;              /* OFX_GN_OPTIMIZE (0): DeformNet.optimize; OFX_GN_ARAP (1): DeformNet.arap */
  int32_t precond_every;     /* the cluster preconditioner is rebuilt on GN steps gn_iter % precond_every == 0
                                (0 or 1: every step) and reused by the warm-started steps in between; it only
                                shapes convergence, the stop test is unchanged */
  double pcg_err_tol;        /* error-based stop (> 0; ABI 5: one Euclidean estimate for every preconditioner): the
                                inner solve also runs until the estimated Euclidean norm of its solution error
                                sqrt(gamma * mu / theta) <= pcg_err_tol (default 2e-6, a fifth of the 1e-5 bar), with
                                gamma = r^T M^-1 r (||e||_A^2 <= gamma / theta), mu = ||p||^2 / p^T A p of the last
                                search direction (||e||_2^2 ~ ||e||_A^2 mu, Hestenes-Stiefel), theta = the smallest
                                Ritz value of the preconditioned operator's Lanczos tridiagonal (from below, within a
                                factor 2^(1/4) down to 2^-10, sqrt 2 below), or, on GN steps after the first, the
                                previous step's final theta when that is smaller; 0: the relative residual alone. Both
                                stop at a relative residual of 1e-12 */
  double precond_rot_tol;    /* adaptive preconditioner refresh (> 0): a GN step also rebuilds the cluster inverse
                                when some node has rotated by more than this (radians, summed |omega| of the
                                steps since the last rebuild); real data with large rotations (the moose demo)
                                needs it, the synthetic bench never reaches it. 0: precond_every alone */
  int32_t precond;           /* PCG preconditioner: OFX_PRECOND_SCHWARZ (1): overlapping additive Schwarz over the
                                8-node clusters extended by up to 16 coupled ring nodes (two launches per PCG
                                iteration, ~3.4x fewer iterations on the bench graph); OFX_PRECOND_CLUSTER (0): the
                                clusters' block Jacobi (one launch per iteration); OFX_PRECOND_AUTO (2, default of the
                                Python API): Schwarz for graphs of >= 1536 nodes, where the cluster blocks' iteration
                                count has grown past what two launches per iteration and the per-solve subdomain
                                inversion cost (config 2's 1020 nodes: 464.7 vs 419.2 frames/s; config 3's 1998:
                                292 vs 378; config 4's 4016: 106.5 vs 159.9). The Schwarz form needs the wave-list PCG
                                (every 8-row wave <= 128 blocks, rows <= 20 blocks) and falls back to the cluster
                                blocks otherwise */
  int32_t _pad1;
} ofx_gn_params;
enum { OFX_PRECOND_CLUSTER = 0, OFX_PRECOND_SCHWARZ = 1, OFX_PRECOND_AUTO = 2 };

/* OFX_GN_ARAP restates DeformNet.arap (model/model.py:1639-1986), the graph-update solve for nodes
 * that are invisible or new: no match rows (n_matches = 0); node_conf = valid-node mask (1/0) and
 * target_node_pos = the valid nodes' targets; per valid node three "flow" rows
 * r = sqrt(lambda_flow)·(g + t - target) whose Jacobian on t is r itself (model.py:1772-1784, as
 * written); ARAP rows as in optimize; only nodes with node_conf == 0 are updated (:1940-1943). With
 * lambda_flow = 0 (model.py:98) the system's exact null space (a common translation of each
 * connected graph component) is projected out of every step, as the dense LU solution has none. */
enum { OFX_GN_OPTIMIZE = 0, OFX_GN_ARAP = 1 };

typedef struct ofx_gn_problem {
  int32_t n_nodes, n_matches, n_neighbors, _pad;
  const float* nodes;           /* (N,3) */
  const int32_t* edges;         /* (N,n_neighbors), -1 padded */
  const float* edge_weights;    /* (N,n_neighbors) or NULL */
  const float* target_node_pos; /* (N,3) motion-complete targets */
  const float* node_conf;       /* (N) */
  const float* src;             /* (M,3) */
  const int32_t* anchors;       /* (M,4) all >= 0 */
  const float* weights;         /* (M,4) */
  const float* tgt;             /* (M,3) */
  const float* target_px;       /* (M) or NULL (only used if lambda_flow != 0) */
  const float* target_py;
  const float* prev_rot;        /* (N,9) or NULL -> identity */
  const float* prev_trans;      /* (N,3) or NULL -> zero */
  float fx, fy, cx, cy;
} ofx_gn_problem;

/* status (device int32[5]): [valid_solve, gn_iterations_accepted, pcg_iterations_total, ill_posed,
 * pcg_capped_steps] — the last: GN steps whose PCG stopped at pcg_max_iter without meeting its stop rule (the step
 * was taken with that iterate)
 * loss_log (device f64[num_iter*4]): per accepted iteration [total, data, arap, motion] */
typedef struct ofx_gn_result {
  float* rot;        /* (N,9) */
  float* trans;      /* (N,3) */
  int32_t* status;
  double* loss_log;
} ofx_gn_result;

/* max_nodes <= 8192 (the JᵀJ slot map is dense over the padded rows) */
int ofx_gn_create(int32_t max_nodes, int32_t max_matches, void** handle);
/* Profiling hook: returns (and resets) the device time of the PCG iteration loops recorded since the
 * last call (hipEvents on the solve stream; synchronises on them), the number of PCG launches (k_pcg_iter
 * launches) and of timed solves; `enable` switches recording for the
 * following steps. */
int ofx_gn_timing(void* handle, int32_t enable, double* pcg_ms, int64_t* iter_launches, int64_t* n_solves);
/* info (host int64[5]) = [n_nodes, n_matches, JᵀJ block count (nnzb), residual terms, rows] of the last
 * setup; rows = nodes in preconditioner-cluster order padded to whole clusters of 8 (<= 2·n_nodes + 8) */
int ofx_gn_info(void* handle, int64_t* info);
/* The preconditioner of the last setup (bench / tools; synchronises the device): info[8] = [Schwarz active, clusters,
 * apply segments (inverse rows of all output clusters), source subdomains, gathered rows, subdomain rows, entries per
 * segment row, kernel launches per PCG iteration (ABI 5: 1 = the one-launch Schwarz iteration k_as_iter, 2 = k_pcg_iter
 * + k_as_apply; 1 for the cluster blocks)]. */
int ofx_gn_precond_info(void* handle, int64_t* info);
/* Waves per PCG cluster workgroup of k_pcg_iter for the last setup (before any: for a small problem): 2 up to
 * 384 clusters (default) or 1 (environment OFX_PCG_W1 set to anything but "" / "0" at create; tuning and A/B
 * only); larger problems always run one wave per cluster. */
int ofx_gn_pcg_waves(void* handle, int32_t* waves);
/* 1 if the last ofx_gn_step's GN update was taken by its converging PCG launch (its stop flag, ofx_gn_stopped, is
 * then already visible to the host when ofx_gn_step returns); 0 if k_step runs as its own launch (the PCG hit
 * pcg_max_iter, or the arap null-space projection runs first): the flag is written asynchronously. */
int ofx_gn_step_fused(void* handle, int32_t* fused);
/* The solve's stop flag as the host sees it (host-mapped, no synchronisation): 1 once a GN step's loss rule
 * (model.py:726-732) or an ill-posed solve stopped it. The device writes it asynchronously: a stepped multi-rank
 * loop reads it only after synchronising the stream behind ofx_gn_step(i), so that every rank leaves after the
 * same step (GaussNewtonSolver.optimize_distributed). */
int ofx_gn_stopped(void* handle, int32_t* stopped);
/* Per-GN-step statistics of the last solve: out (host f64[3*cap]) = [PCG iterations, |b|², loss] per
 * step (zeros for steps that did not run); synchronous D2H copy, at most 64 steps. */
int ofx_gn_stats(void* handle, double* out, int32_t cap);
/* Row order of the last setup: perm (host int32[cap]) = node of each PCG row, -1 for padding rows
 * (the order of rhs and of the solver's per-node state); cap must be >= rows (ofx_gn_info()[4]). */
int ofx_gn_row_order(void* handle, int32_t* perm, int32_t cap);
int ofx_gn_destroy(void* handle);
/* Upload + build the block-sparse JᵀJ pattern (co-anchored node pairs, edges, diagonal).
 * Copies nodes/edges to the host (one stream sync) to order the rows by graph clusters when the
 * graph changed, and synchronises once more to size the pattern; *nnz_blocks receives the block count. */
int ofx_gn_setup(void* handle, const ofx_gn_problem* prob, const ofx_gn_params* params, int64_t* nnz_blocks,
                 ofx_stream_t s);
/* Assemble A (f64[nnz_blocks*36]) and rhs (f64[6·rows+4]: b = -Jᵀr then [loss² total,data,arap,motion])
 * from matches [m0,m1); regularizers (ARAP, motion) and the LM damping λ_k·I of the diagonal blocks
 * (model.py:418-419,641-662) added iff add_reg. Zeroes both first.
 * In a multi-GPU solve every rank calls this on its match shard, the caller all-reduces
 * (sum) A and rhs, then every rank calls ofx_gn_step with identical buffers. */
int ofx_gn_linearize(void* handle, int32_t gn_iter, int32_t m0, int32_t m1, int32_t add_reg, double* A,
                     double* rhs, ofx_stream_t s);
/* Cluster block-Jacobi PCG solve of A x = b, early-stop bookkeeping, R <- exp(x_rot) R, t += x_t. */
int ofx_gn_step(void* handle, int32_t gn_iter, double* A, double* rhs, ofx_stream_t s);
int ofx_gn_finish(void* handle, const ofx_gn_result* res, ofx_stream_t s);
/* setup + num_iter x (linearize + step) + finish, single device */
int ofx_gn_solve(void* handle, const ofx_gn_problem* prob, const ofx_gn_params* params,
                 const ofx_gn_result* res, ofx_stream_t s);
/* Prefetch the setup of the NEXT problem on this handle (software pipelining across frames; no reference
 * twin — the reference sets up every solve inline, model.py:222-415). Returns at once: the setup (upload,
 * JᵀJ pattern, contribution lists, with its one host sync) runs on a host thread and on the handle's own
 * stream, ordered after everything enqueued on `s` so far, concurrently with the caller's other work (the
 * current frame's solve on another handle). The following ofx_gn_solve on this handle with the same problem
 * (same buffers and sizes, same params; prev_rot / prev_trans may differ: they are read by the solve)
 * skips its setup, waits for the prefetched one on its own stream and loads the pose. A different problem,
 * or a prefetch that failed, falls back to the inline setup. The problem's buffers must stay allocated and
 * unchanged until that solve. */
int ofx_gn_prepare(void* handle, const ofx_gn_problem* prob, const ofx_gn_params* params, ofx_stream_t s);
/* ofx_gn_prepare, started later: the prefetch's host thread waits until the next ofx_gn_solve on `trigger`
 * (another handle) has queued the first kernels of GN step `gn_step`, or returns, or ofx_gn_prepare_wait /
 * ofx_gn_solve / ofx_gn_destroy on this handle needs it. The setup's kernels then overlap that solve's last steps
 * instead of following them. The ordering on `s` is taken now, as for ofx_gn_prepare. */
int ofx_gn_prepare_after(void* handle, const ofx_gn_problem* prob, const ofx_gn_params* params, ofx_stream_t s,
                         void* trigger, int32_t gn_step);
/* Wait (host) until a prefetch on this handle has been enqueued, and order stream `s` after it: a
 * synchronisation of `s` afterwards covers the prefetched setup. */
int ofx_gn_prepare_wait(void* handle, ofx_stream_t s);
/* Make `handle` use `other`'s per-GN-step PCG iteration history (it sizes the first chunk of iteration
 * launches; results do not depend on it): the solver slots of one frame loop then predict from the previous
 * frame whichever slot solved it. */
int ofx_gn_share_history(void* handle, void* other);
/* Solves on this handle that used a prefetched setup / discarded one (a different problem or a failure). */
int ofx_gn_prefetch_stats(void* handle, int64_t* used, int64_t* missed);
/* Host work to run once inside the next solve on this handle, while its host loop waits for the first GN step's PCG
 * chunk (the host is otherwise idle there): fn(arg) is called on the solving thread, then forgotten; NULL fn clears a
 * pending one. A frame loop uses it to enqueue the previous frame's integrate (on a stream of its own) without holding
 * back the next solve's first launches. (Round 6; no ABI struct changes.) */
int ofx_gn_set_idle_hook(void* handle, void (*fn)(void*), void* arg);

#ifdef __cplusplus
}
#endif
#endif /* OFX_H */
