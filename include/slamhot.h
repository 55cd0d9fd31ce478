/*
 * slamhot.h — C-ABI of the MI355X-native ORB-SLAM3 hot path (gfx950, HIP).
 *
 * This is the drop-in boundary.  Every entry point replaces one reference interface;
 * the citation after each declaration names it (paths relative to the ORB-SLAM3-Noted
 * reference tree).  Conventions:
 *   - plain C types only: pointers + sizes, no C++ / OpenCV / torch types;
 *   - the caller owns every host buffer; a handle owns its device memory and a private
 *     HIP stream;
 *   - every call returns a slam_status; negative = error; nothing throws across the ABI;
 *   - handles are independent (thread-safe across handles, not within one handle),
 *     mirroring "one ORBextractor per camera, used by one thread at a time"
 *     (Frame.cc:119-122).
 *   - there is no CPU fallback: without a usable gfx950 device, create() fails with
 *     SLAM_ENODEV.
 */
#ifndef SLAMHOT_H
#define SLAMHOT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t slam_status;
enum {
    SLAM_OK = 0,
    SLAM_EINVAL = -1,  /* bad argument / shape */
    SLAM_ENOMEM = -2,  /* device or host allocation failed */
    SLAM_EHIP = -3,    /* HIP runtime error */
    SLAM_ECAP = -4,    /* output capacity too small (n holds the required size) */
    SLAM_ENODEV = -5,  /* no gfx950 device */
    SLAM_EEMPTY = -6,  /* empty image (reference returns -1, ORBextractor.cc:1072-1073) */
    SLAM_ETIMEDOUT = -7 /* a bounded wait expired (host wait on device progress, or a device-side
                           hand-off wait); the handle's stream state is printed on stderr */
};

/* cv::KeyPoint memory layout (28 bytes): pt.x, pt.y, size, angle, response, octave, class_id */
typedef struct slam_keypoint {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} slam_keypoint;

/* ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
 * (ORBextractor.h:49-50, ORBextractor.cc:408-468) */
typedef struct slam_orb_params {
    int32_t nfeatures;
    float scale_factor;
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
} slam_orb_params;

typedef struct slam_extractor slam_extractor;

/* Library / device probing. */
const char* slamhot_version(void);
const char* slamhot_status_string(slam_status s);
slam_status slamhot_device_count(int* n);

/* ---------------------------------------------------------------------------------
 * ORB extractor
 * ------------------------------------------------------------------------------- */

/* Replaces ORBextractor::ORBextractor (ORBextractor.cc:408-468).  max_width/max_height
 * bound the frames; max_batch bounds slamhot_extract_batch*.  The scale tables are built
 * on the host exactly as the reference builds them. */
slam_status slamhot_extractor_create(const slam_orb_params* params, int device, int max_width,
                                     int max_height, int max_batch, slam_extractor** out);
void slamhot_extractor_destroy(slam_extractor* ex);

/* Replaces GetLevels/GetScaleFactors/GetInverseScaleFactors/GetScaleSigmaSquares/
 * GetInverseScaleSigmaSquares (ORBextractor.h:61-81) and the private mnFeaturesPerLevel.
 * Each array has nlevels entries; any pointer may be NULL. */
slam_status slamhot_extractor_levels(const slam_extractor* ex, int* nlevels, float* scale,
                                     float* inv_scale, float* sigma2, float* inv_sigma2,
                                     int32_t* nfeatures_per_level);

/* Replaces int ORBextractor::operator()(img, mask, keypoints, descriptors, vLappingArea)
 * (ORBextractor.cc:1068-1150) for ONE host image (CV_8UC1, row stride `stride` bytes).
 * Writes up to `cap` keypoints (cv::KeyPoint layout) and cap*32 descriptor bytes, in the
 * reference's output order (level-major, octree order, lapping split from the back).
 * *n = number of keypoints, *mono_index = operator()'s return value.  Returns SLAM_ECAP
 * (with *n set) if cap is too small. */
slam_status slamhot_extract(slam_extractor* ex, const uint8_t* img, int width, int height,
                            size_t stride, int lap0, int lap1, slam_keypoint* kps,
                            uint8_t* desc, int cap, int* n, int* mono_index);

/* Batched form: nframes host images of identical size, frame f at img + f*height*stride.
 * Outputs are strided by cap per frame: kps[f*cap + i], desc[(f*cap + i)*32].  n and
 * mono_index have nframes entries. */
slam_status slamhot_extract_batch(slam_extractor* ex, int nframes, const uint8_t* imgs,
                                  int width, int height, size_t stride, int lap0, int lap1,
                                  slam_keypoint* kps, uint8_t* desc, int cap, int* n,
                                  int* mono_index);

/* Device-resident batch (inputs already in HBM).  d_imgs: nframes*height*width bytes
 * (tight rows).  Outputs are device pointers with the same layout as the host batch form.
 * `hip_stream` may be NULL (the handle's stream).  Asynchronous: synchronise the stream
 * before reading outputs.  Capacity overflow is reported per frame by n[f] > cap. */
slam_status slamhot_extract_batch_device(slam_extractor* ex, int nframes, const void* d_imgs,
                                         int width, int height, int lap0, int lap1,
                                         void* d_kps, void* d_desc, int cap, void* d_n,
                                         void* d_mono_index, void* hip_stream);

/* Public ORBextractor::mvImagePyramid (ORBextractor.h:83), read by
 * Frame::ComputeStereoMatches: copies level `level` of batch frame `frame` of the last
 * extraction into dst (tight rows, capacity dst_cap bytes) and returns its size. */
slam_status slamhot_pyramid_level(slam_extractor* ex, int frame, int level, uint8_t* dst,
                                  size_t dst_cap, int* width, int* height);

/* Device view of the same level (no copy): pointer, row pitch, size.  Valid until the next
 * extraction on this handle; level 0 is the caller's device input for extract_batch_device. */
slam_status slamhot_pyramid_level_device(slam_extractor* ex, int frame, int level, const void** d_ptr,
                                         int* pitch, int* width, int* height);

/* Stream the handle works on (hipStream_t as void*). */
void* slamhot_extractor_stream(slam_extractor* ex);

/* Measurement hooks (no reference counterpart; the reference's REGISTER_TIMES timers,
 * Config.h:4 / Frame.cc:116-127, play this role there).  With profiling on, every stage
 * of every launch is bracketed by HIP events on the launch stream; stage_stats syncs on
 * them and returns per-stage accumulated milliseconds and launch counts
 * (slamhot_extractor_num_stages() entries each). */
slam_status slamhot_extractor_set_profiling(slam_extractor* ex, int enable);
int slamhot_extractor_num_stages(void);
const char* slamhot_extractor_stage_name(int stage);
slam_status slamhot_extractor_stage_stats(slam_extractor* ex, double* total_ms, long* launches,
                                          int reset);

/* ---------------------------------------------------------------------------------
 * Frame construction after extraction (monocular / RGB-D / unrectified cameras)
 * ------------------------------------------------------------------------------- */
/* void Frame::UndistortKeyPoints() (Frame.cc:730-763): mvKeysUn = cv::undistortPoints(mvKeys,
 * K, mDistCoef, R = I, P = mK) with OpenCV 4.2.0's default 5 iterations.  K = (fx, fy, cx, cy)
 * of the Pinhole camera (toK() and mK are the same matrix), dist = mDistCoef (k1, k2, p1, p2
 * [, k3]), ndist 4 or 5 (0, or dist[0] == 0: mvKeysUn = mvKeys).  Every keypoint field but pt
 * is copied.  Host buffers, synchronous. */
slam_status slamhot_undistort_keypoints(int device, const float* K, const float* dist, int ndist, int n,
                                        const slam_keypoint* kps, slam_keypoint* kps_un);
/* The same for nframes frames left in HBM by slamhot_extract_batch_device (d_kps cap per frame,
 * d_n per frame) into d_kps_un (cap per frame); asynchronous on hip_stream. */
slam_status slamhot_undistort_keypoints_batch_device(const float* K, const float* dist, int ndist, int nframes,
                                                     const void* d_kps, const void* d_n, int cap, void* d_kps_un,
                                                     void* hip_stream);
/* void Frame::ComputeImageBounds(const cv::Mat&) (Frame.cc:765-792): bounds = (mnMinX, mnMaxX,
 * mnMinY, mnMaxY) from the undistorted image corners (the image size without distortion). */
slam_status slamhot_image_bounds(const float* K, const float* dist, int ndist, int cols, int rows, float* bounds);

/* ---------------------------------------------------------------------------------
 * Vocabulary (DBoW2 TemplatedVocabulary<FORB>, ORBVocabulary.h:29-30)
 * ------------------------------------------------------------------------------- */
typedef struct slam_vocab slam_vocab;

/* Node table in DBoW2 order: node 0 is the root; parent[0] = -1.  Children of a node are
 * the nodes naming it as parent, in table order (loadFromTextFile, TemplatedVocabulary.h:
 * 1350-1436).  is_leaf marks words; weight is the node weight (word idf). */
slam_status slamhot_vocab_create(int device, int k, int L, int scoring, int weighting, int n_nodes,
                                 const int32_t* parent, const uint8_t* is_leaf,
                                 const uint8_t* desc, const double* weight, slam_vocab** out);
/* TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1350-1436), ORBvoc.txt. */
slam_status slamhot_vocab_load_text(int device, const char* path, slam_vocab** out);
void slamhot_vocab_destroy(slam_vocab* v);
slam_status slamhot_vocab_info(const slam_vocab* v, int* k, int* L, int* n_nodes, int* n_words);

/* TemplatedVocabulary::transform(desc, word_id, weight, &node_id, levelsup) for n
 * descriptors (TemplatedVocabulary.h:1229-1271); the per-feature results from which
 * Frame::ComputeBoW / KeyFrame::ComputeBoW (Frame.cc:721-728) build mBowVec/mFeatVec
 * (features with weight <= 0 are dropped, :1169). */
slam_status slamhot_vocab_transform(slam_vocab* v, int n, const uint8_t* desc, int levelsup,
                                    int32_t* word_id, double* weight, int32_t* node_id);
/* void TemplatedVocabulary::transform(const vector<TDescriptor>& features, BowVector& v,
 * FeatureVector& fv, int levelsup) (TemplatedVocabulary.h:1139-1206), the whole body of
 * Frame::ComputeBoW / KeyFrame::ComputeBoW (Frame.cc:721-728, KeyFrame.cc:105-114): the descent of
 * every descriptor on the device, then DBoW2's BowVector and FeatureVector on the host exactly as
 * the reference builds them — features whose word weight is <= 0 dropped (:1169); TF_IDF / TF:
 * BowVector::addWeight (sum in feature order), divided by the word count when the scoring does not
 * normalise (:1174-1180); IDF / BINARY: addIfNotExist (first weight, :1195); then the scoring's
 * L1 / L2 normalisation (BowVector.cpp:62-84; L1 for L1 / chi-square / KL / Bhattacharyya, none for
 * dot product).  Outputs, caller-owned with room for n entries (n + 1 for fv_off):
 *   BowVector:     *n_words pairs (bow_word ascending, bow_value)
 *   FeatureVector: *n_nodes nodes (fv_node ascending), node j's features fv_feat[fv_off[j] ..
 *                  fv_off[j+1]) ascending (FeatureVector::addFeature, FeatureVector.cpp:31-45). */
slam_status slamhot_compute_bow(slam_vocab* v, int n, const uint8_t* desc, int levelsup, int* n_words,
                                uint32_t* bow_word, double* bow_value, int* n_nodes, uint32_t* fv_node,
                                int32_t* fv_off, uint32_t* fv_feat);
/* Device-resident form: d_desc n x 32 (row stride desc_stride bytes), outputs on device. */
slam_status slamhot_vocab_transform_device(slam_vocab* v, int n, const void* d_desc,
                                           int desc_stride, int levelsup, void* d_word_id,
                                           void* d_weight, void* d_node_id, void* hip_stream);

/* ---------------------------------------------------------------------------------
 * ORBmatcher (ORBmatcher.h:39-91), pinhole cameras (Frame::Nleft == -1)
 * ------------------------------------------------------------------------------- */
typedef struct slam_matcher slam_matcher;

slam_status slamhot_matcher_create(int device, slam_matcher** out);
void slamhot_matcher_destroy(slam_matcher* m);
/* Timing of the handle's last batched host-buffer call (slamhot_search_local_points_batch,
 * slamhot_search_by_projection_{last,kf}_batch), from events on its stream: kernel_ms = the
 * call's kernels, span_ms = first upload to the end of the read-back (device side). */
slam_status slamhot_matcher_last_batch_stats(const slam_matcher* m, float* kernel_ms, float* span_ms);

/* One side of SearchByBoW: descriptors, keypoint angles, MapPoint validity
 * (pMP != NULL && !pMP->isBad(); NULL = all valid) and the DBoW2 FeatureVector as CSR
 * (node ids ascending, feature indices ascending inside each node). */
typedef struct slam_bow_side {
    int32_t n;
    const uint8_t* desc;
    const float* angle;
    const uint8_t* valid;
    int32_t n_nodes;
    const uint32_t* node_id;
    const int32_t* node_off;
    const uint32_t* node_feat;
} slam_bow_side;

/* int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& matches)
 * (ORBmatcher.cc:269-471) when strict == 0: A = KF (valid = MapPoint flags), B = Frame
 * (valid NULL); b2a[i] = KF feature whose MapPoint F.feature i matched, -1 otherwise.
 * int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& m12)
 * (ORBmatcher.cc:823-963) when strict == 1: a2b[i] = KF2 feature matched by KF1 feature i.
 * *nmatches = the reference's return value. */
slam_status slamhot_search_by_bow(slam_matcher* m, const slam_bow_side* A, const slam_bow_side* B,
                                  float nnratio, int check_ori, int strict, int32_t* a2b,
                                  int32_t* b2a, int* nmatches);

/* ---------------------------------------------------------------------------------
 * SearchByProjection (pinhole, Nleft == -1).  The current Frame as the matchers read it.
 * ------------------------------------------------------------------------------- */
typedef struct slam_frame_view {
    int32_t n;
    const slam_keypoint* kps_un;  /* mvKeysUn (pt, octave, angle) */
    const float* uright;          /* mvuRight, -1 = no stereo; NULL = all -1 */
    const uint8_t* desc;          /* mDescriptors, n x 32 */
    const int8_t* mp_state;       /* mvpMapPoints on entry: -1 empty, 0 MapPoint without
                                     observations, 1 MapPoint with Observations() > 0 */
    float min_x, min_y, max_x, max_y;   /* mnMinX.. (Frame::ComputeImageBounds) */
    float grid_inv_w, grid_inv_h;       /* mfGridElementWidthInv / HeightInv */
    int32_t nlevels;
    const float* scale;           /* mvScaleFactors */
    float log_scale;              /* mfLogScaleFactor */
    float fx, fy, cx, cy, bf, b;  /* Pinhole parameters, mbf, mb */
    const float* Tcw;             /* 4x4 row-major float pose (B4, B6); NULL for B5 */
} slam_frame_view;

/* Per local MapPoint, the tracking fields Frame::isInFrustum (Frame.cc:493-570) leaves. */
typedef struct slam_mp_track {
    float proj_x, proj_y, proj_xr, depth, view_cos;
    int32_t scale_level;
    uint8_t in_view, is_bad, has_obs, pad;
} slam_mp_track;

/* int SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, float th,
 * bool bFarPoints, float thFarPoints) (ORBmatcher.cc:44-214).  f_match[i] = index of the
 * MapPoint this call assigned to F feature i (the last assignment wins, as in the
 * reference), -1 if untouched. */
slam_status slamhot_search_by_projection_local(slam_matcher* m, const slam_frame_view* F, int n_mp,
                                               const slam_mp_track* mps, const uint8_t* mp_desc,
                                               float nnratio, float th, int far_points,
                                               float th_far, int32_t* f_match, int* nmatches);

/* One local MapPoint as Tracking::SearchLocalPoints sees it (Tracking.cc:3213-3231). */
typedef struct slam_mp_geom {
    float pos[3];                 /* GetWorldPos2 (mWorldPosx) */
    float normal[3];              /* GetNormal2 (mNormalVectorx) */
    float min_dist, max_dist;     /* mfMinDistance, mfMaxDistance (the 0.8f / 1.2f invariance
                                     factors of GetMin/MaxDistanceInvariance are applied here) */
    uint8_t seen;                 /* mnLastFrameSeen == mCurrentFrame.mnId (already matched) */
    uint8_t is_bad;               /* isBad() */
    uint8_t has_obs;              /* Observations() > 0 */
    uint8_t pad;
} slam_mp_geom;

/* Tracking::SearchLocalPoints' second half (Tracking.cc:3213-3258) for a Frame with
 * Nleft == -1: Frame::isInFrustum(pMP, view_cos_limit) (Frame.cc:493-556, with
 * MapPoint::PredictScale, MapPoint.cc:551-566) for every MapPoint not seen / not bad, then, when
 * any is in view, SearchByProjection(F, vpMapPoints, th, bFarPoints, thFarPoints)
 * (ORBmatcher.cc:44-214) — both on the device, no host round trip between them.  F->Tcw is
 * required.  Outputs: f_match / nmatches as slamhot_search_by_projection_local; *n_to_match =
 * the number of MapPoints isInFrustum accepted; track (optional, n_mp) = the tracking fields
 * isInFrustum leaves (in_view = mbTrackInView). */
slam_status slamhot_search_local_points(slam_matcher* m, const slam_frame_view* F, int n_mp,
                                        const slam_mp_geom* mps, const uint8_t* mp_desc, float view_cos_limit,
                                        float nnratio, float th, int far_points, float th_far,
                                        slam_mp_track* track, int* n_to_match, int32_t* f_match, int* nmatches);

/* Batched form of slamhot_search_local_points: nframes independent (Frame, local map) problems
 * (frames[f] with n_mp[f] MapPoints mps[f] / mp_desc[f]) in one upload and two launches (one
 * isInFrustum grid row and one SearchByProjection workgroup per frame).  Outputs per frame:
 * f_match[f] (frames[f].n entries), n_to_match[f], nmatches[f]; identical to nframes single calls. */
slam_status slamhot_search_local_points_batch(slam_matcher* m, int nframes, const slam_frame_view* frames,
                                              const int32_t* n_mp, const slam_mp_geom* const* mps,
                                              const uint8_t* const* mp_desc, float view_cos_limit, float nnratio,
                                              float th, int far_points, float th_far, int32_t* const* f_match,
                                              int32_t* n_to_match, int32_t* nmatches);

/* The previous Frame for SearchByProjection(Frame&, const Frame& LastFrame, th, bMono)
 * (ORBmatcher.cc:2173-2389): per last-frame feature its MapPoint (has_mp, outlier flag,
 * world position, descriptor, Observations()>0) and keypoint octave/angle. */
typedef struct slam_last_frame {
    int32_t n;
    const float* Tcw;             /* 4x4 row-major */
    const slam_keypoint* kps;     /* mvKeys (octave) */
    const slam_keypoint* kps_un;  /* mvKeysUn (angle) */
    const uint8_t* has_mp;
    const uint8_t* outlier;       /* mvbOutlier */
    const float* mp_pos;          /* n x 3 world position */
    const uint8_t* mp_desc;       /* n x 32 */
    const uint8_t* mp_has_obs;
} slam_last_frame;

/* f_match[i] (F->n entries) for this and slamhot_search_by_projection_kf: the LastFrame / KeyFrame
 * feature whose MapPoint this call wrote into CurrentFrame.mvpMapPoints[i] (the last assignment
 * wins), -1 if the call left entry i untouched, -2 if it assigned entry i and the rotation check
 * then set it to NULL (ORBmatcher.cc:2366-2386, 2491-2510: that NULL overwrites whatever the entry
 * held before the call). */
slam_status slamhot_search_by_projection_last(slam_matcher* m, const slam_frame_view* F,
                                              const slam_last_frame* LF, float nnratio, int check_ori,
                                              float th, int mono, int32_t* f_match, int* nmatches);

/* Batched, device-resident Frame::ComputeBoW + SearchByBoW(KeyFrame*, Frame&) (ORBmatcher.cc:
 * 269-471; strict = 1 gives the KF-KF acceptance of :823-963) over frame pairs, for
 * extraction output left in HBM by slamhot_extract_batch_device: d_kps (nframes x cap
 * slam_keypoint), d_desc (nframes x cap x 32), d_n (nframes int32).  Every frame's
 * FeatureVector at level L-levelsup is built on the device (TemplatedVocabulary.h:1139-1206,
 * FeatureVector.cpp:31-45).  pairs (host, 2 x npairs): (keyframe index, frame index).
 * d_valid (nframes x cap u8, may be NULL = all valid) marks keyframe features with a usable
 * MapPoint.  Outputs (device, cap per pair): d_a2b, d_b2a (-1 = none), d_nmatches (npairs).
 * cap <= 8192.  Asynchronous on hip_stream (NULL = the matcher's stream).  Every pair's outputs
 * are defined: a pair outside the fast kernel's tiles (a side over 8192 features or 4096 nodes,
 * or a frame node over 256 candidates) runs through an unbounded kernel with the same results;
 * slamhot_bow_match_batch_status synchronises and reports how many pairs took that path. */
slam_status slamhot_bow_match_batch_device(slam_matcher* m, slam_vocab* v, int nframes, const void* d_kps,
                                           const void* d_desc, int cap, const void* d_n, const void* d_valid,
                                           int npairs, const int32_t* pairs, float nnratio, int check_ori,
                                           int strict, int levelsup, void* d_a2b, void* d_b2a,
                                           void* d_nmatches, void* hip_stream);
slam_status slamhot_bow_match_batch_status(slam_matcher* m, void* hip_stream, int* general_pairs);

/* Per KeyFrame feature for SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&
 * sAlreadyFound, float th, int ORBdist) (ORBmatcher.cc:2391-2513). */
typedef struct slam_kf_points {
    int32_t n;
    const slam_keypoint* kps_un;  /* KF mvKeysUn (angle) */
    const uint8_t* use;           /* MapPoint present, !isBad, not in sAlreadyFound */
    const float* mp_pos;          /* n x 3 */
    const float* max_dist;        /* mfMaxDistance */
    const float* min_dist;        /* mfMinDistance */
    const uint8_t* mp_desc;       /* n x 32 */
} slam_kf_points;

slam_status slamhot_search_by_projection_kf(slam_matcher* m, const slam_frame_view* F,
                                            const slam_kf_points* KF, float nnratio, int check_ori,
                                            float th, int orb_dist, int32_t* f_match, int* nmatches);

/* Batched forms of the two projection matchers above: nframes independent problems staged into
 * one pinned host image, one upload, one k_search_by_projection launch (a workgroup per frame),
 * one copy back; results identical to nframes single calls.  f_match[f] holds frames[f].n
 * entries, nmatches[f] the count.
 *   _last_batch: SearchByProjection(Frame&, const Frame& LastFrame, th, bMono), the matcher of
 *     Tracking::TrackWithMotionModel, which every steady-state frame runs (Tracking.cc:2683-2760,
 *     ORBmatcher.cc:2173-2389); frame f against last[f].
 *   _kf_batch: SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)
 *     (Tracking::Relocalization, Tracking.cc:3455-3590; ORBmatcher.cc:2391-2513); frame f
 *     against kfs[f]. */
slam_status slamhot_search_by_projection_last_batch(slam_matcher* m, int nframes, const slam_frame_view* frames,
                                                    const slam_last_frame* last, float nnratio, int check_ori,
                                                    float th, int mono, int32_t* const* f_match, int32_t* nmatches);
slam_status slamhot_search_by_projection_kf_batch(slam_matcher* m, int nframes, const slam_frame_view* frames,
                                                  const slam_kf_points* kfs, float nnratio, int check_ori,
                                                  float th, int orb_dist, int32_t* const* f_match, int32_t* nmatches);

/* ------------------------------------------------------------------------------------------
 * Local bundle adjustment: the g2o LM/Schur solve inside
 *   static void Optimizer::LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag, Map* pMap,
 *       int& num_fixedKF, int& num_OptKF, int& num_MPs, int& num_edges)
 *   (Optimizer.h:59, Optimizer.cc:1611-2078).
 * The caller (the shim in INTEGRATION.md) builds the window exactly as Optimizer.cc:1613-1718
 * does and flattens it: KeyFrames in vertex-id (mnId) order, MapPoints in lLocalMapPoints
 * order, edges in insertion order (point-major: the edges of one MapPoint are contiguous,
 * Optimizer.cc:1801-1920).  The solver then runs the reference schedule on the device:
 * optimize(5) -> [stop flag] -> initializeOptimization(0) + optimize(10) (:1925-1987), and
 * classifies the final outliers (chi2 > 5.991 mono / 7.815 stereo, or depth <= 0,
 * :1995-2038).  The caller erases those observations and writes poses/points back
 * (:2041-2077).  Many independent windows may be solved in one call (batched mode).
 * ------------------------------------------------------------------------------------------ */

/* KeyFrame intrinsics used by the edges: fx, fy, cx, cy, mbf (KeyFrame.h float members;
 * Pinhole mvParameters for the mono edge, EdgeStereoSE3ProjectXYZ::fx.. for stereo). */
typedef struct slam_camera {
    float fx, fy, cx, cy, bf;
} slam_camera;

typedef struct slam_lba_problem {
    int32_t n_kf;               /* KeyFrame vertices (local + fixed), mnId order */
    const float* kf_Tcw;        /* n_kf x 16, row-major KeyFrame::GetPose() (cv::Mat 4x4 f32) */
    const uint8_t* kf_fixed;    /* 0 free, 1 the map init KF (setFixed, written back), 2 lFixedCameras */
    int32_t n_pt;               /* MapPoint vertices (all marginalized) */
    const float* pt_pos;        /* n_pt x 3, MapPoint::GetWorldPos() */
    int32_t n_edge;             /* edges, insertion order, edge_pt non-decreasing */
    const int32_t* edge_pt;     /* vertex 0: MapPoint index */
    const int32_t* edge_kf;     /* vertex 1: KeyFrame index */
    const float* edge_obs;      /* n_edge x 3: kpUn.pt.x, kpUn.pt.y, mvuRight (< 0 -> mono) */
    const float* edge_inv_sigma2; /* mvInvLevelSigma2[kpUn.octave] */
    slam_camera cam;
    double user_lambda_init;    /* this window's pMap: > 0 sets the initial LM lambda (100 when
                                   pMap->IsInertial(), Optimizer.cc:1726-1727); 0 -> the options value */
    /* Right-camera observations of KeyFrames with a second camera (pKFi->mpCamera2, pinhole
     * here): EdgeSE3ProjectXYZToBody (OptimizableTypes.h:117-144, OptimizableTypes.cpp:192-215),
     * inserted by Optimizer.cc:1883-1914 right after the KeyFrame's left edge.  NULL = none. */
    const uint8_t* edge_body;   /* n_edge: 1 = body edge (edge_obs = mvKeysRight[..].pt, [2] unused;
                                   inv_sigma2 of that keypoint's octave; Huber / chi2 as mono) */
    const float* kf_Trl;        /* n_kf x 16 row-major KeyFrame::mTrl (right <- left), read for KFs
                                   with body edges (Converter::toSE3Quat) */
    slam_camera cam2;           /* mpCamera2 parameters fx, fy, cx, cy (bf unused) */
    /* A camera per KeyFrame: the reference binds every edge to its own KeyFrame's calibration
     * (mono e->pCamera = pKFi->mpCamera, Optimizer.cc:1840; stereo e->fx..bf = pKFi->fx..mbf,
     * :1869-1873; body e->pCamera = pKFi->mpCamera2, :1906), so one window (an Atlas map built
     * from several cameras) and one batch may mix calibrations.  NULL = cam / cam2 for every
     * KeyFrame of this window. */
    const slam_camera* kf_cam;  /* n_kf: pKFi->fx, fy, cx, cy, mbf */
    const slam_camera* kf_cam2; /* n_kf: pKFi->mpCamera2 fx, fy, cx, cy (read for KFs with body edges) */
} slam_lba_problem;

typedef struct slam_lba_options {
    int32_t iters_first;        /* 5  (Optimizer.cc:1926) */
    int32_t iters_second;       /* 10 (Optimizer.cc:1986) */
    double user_lambda_init;    /* 0 -> tau * max diag(H); 100 if pMap->IsInertial() (:1726) */
    const volatile uint8_t* stop_flag_bool; /* optional: the caller's `bool* pbStopFlag` itself (a C++
                                   bool is one byte), polled live like the int32 stop_flag */
    /* optional diagnostic hook (NULL = none): called on the calling thread each time the host has
     * seen the counters of an LM step, with the step's number (0-based over the whole call).  A
     * hook that sets the stop flag at step k stops the solve within the steps already queued
     * behind k (at most 3 more: the host keeps a ring of 4 steps in flight), the same bound
     * g2o's asynchronous terminate() check has; the step it lands on depends on timing. */
    void (*step_hook)(void* ctx, int32_t step);
    void* step_hook_ctx;
} slam_lba_options;

typedef struct slam_lba_result {
    float* kf_Tcw;              /* out n_kf x 16 (fixed KFs are copied through) */
    float* pt_pos;              /* out n_pt x 3 */
    uint8_t* edge_outlier;      /* out n_edge: 1 = goes to vToErase (Optimizer.cc:1995-2038) */
    int32_t iterations[2];      /* LM iterations run by each optimize() call */
    int32_t trials;             /* total LM trials (linear solves) */
    int32_t n_outlier;
    double chi2_initial;        /* activeRobustChi2 at the first iteration */
    double chi2_final;          /* activeRobustChi2 after the last accepted step */
    double lambda_final;
    int32_t ran;                /* 0: the stop flag was already set on entry, nothing was optimized
                                   and nothing is to be written back (Optimizer.cc:1921-1923) */
} slam_lba_result;

typedef struct slam_lba slam_lba;

/* A solver handle keeps device buffers sized for the largest batch seen (grown on demand). */
slam_status slamhot_lba_create(int device, slam_lba** out);
void slamhot_lba_destroy(slam_lba* s);
/* Solve n_prob independent windows.  stop_flag (may be NULL; or options->stop_flag_bool) is the
 * pbStopFlag, and it is LIVE: the calling thread polls it while the device works and mirrors it
 * into pinned memory that the LM control kernel reads at the end of every trial, so a flag set
 * by another thread during the solve (LocalMapping.cc:300 mbAbortBA) ends every window's
 * optimize() at its next trial, as SparseOptimizer::terminate() does (sparse_optimizer.h:188,
 * sparse_optimizer.cpp:376, optimization_algorithm_levenberg.cpp:149); a flag set before the call
 * returns at once with nothing written back but the copied inputs (Optimizer.cc:1921-1923), and one
 * set during the first optimize(5) skips the second (Optimizer.cc:1933-1935). */
slam_status slamhot_lba_solve(slam_lba* s, int n_prob, const slam_lba_problem* probs,
                              const slam_lba_options* opt, const volatile int32_t* stop_flag,
                              slam_lba_result* results);
/* Warm a handle for windows of about n_kf KeyFrames x n_pt MapPoints x obs_per_pt observations:
 * one synthetic window of that size is solved, which loads every kernel of the single-window path
 * and sizes the device buffers and the pinned staging arena, so LocalMapping's first
 * LocalBundleAdjustment (LocalMapping.cc:161) costs what every later one does. */
slam_status slamhot_lba_warmup(slam_lba* s, int n_kf, int n_pt, int obs_per_pt);
/* Last solve: device time (ms, kernels + copies), host plan time (ms: graph structure build
 * and upload, buildStructure in g2o), and the number of host<->device round trips. */
slam_status slamhot_lba_last_stats(const slam_lba* s, double* device_ms, double* plan_ms, int* syncs);

/* ------------------------------------------------------------------------------------------
 * Motion-only BA: int Optimizer::PoseOptimization(Frame* pFrame) (Optimizer.h:55,
 * Optimizer.cc:824-1118), pinhole (no mpCamera2).  Four rounds of optimize(10) from the
 * frame's initial pose, each re-classifying every observation by chi2 (5.991 mono / 7.815
 * stereo) and excluding outliers from the next round; the Huber kernel is dropped after the
 * third round.  Batched: one workgroup per frame.
 * ------------------------------------------------------------------------------------------ */
typedef struct slam_pose_frame {
    float Tcw[16];               /* pFrame->mTcw, row-major 4x4 */
    int32_t n;                   /* pFrame->N */
    const slam_keypoint* kps_un; /* mvKeysUn: x, y, octave used */
    const float* uright;         /* mvuRight (< 0 -> monocular observation) */
    const uint8_t* has_mp;       /* mvpMapPoints[i] != NULL */
    const float* mp_pos;         /* n x 3 MapPoint::GetWorldPos (read where has_mp) */
    const float* inv_sigma2;     /* mvInvLevelSigma2 */
    int32_t nlevels;
    slam_camera cam;
} slam_pose_frame;

typedef struct slam_pose_result {
    float Tcw[16];               /* pFrame->SetPose (input pose when fewer than 3 observations) */
    uint8_t* outlier;            /* n: pFrame->mvbOutlier (only entries with has_mp are written) */
    int32_t n_initial;           /* nInitialCorrespondences */
    int32_t n_inliers;           /* return value: nInitialCorrespondences - nBad (0 if < 3) */
} slam_pose_result;

typedef struct slam_pose_opt slam_pose_opt;
slam_status slamhot_pose_opt_create(int device, slam_pose_opt** out);
void slamhot_pose_opt_destroy(slam_pose_opt* h);
slam_status slamhot_pose_optimization(slam_pose_opt* h, int nframes, const slam_pose_frame* frames,
                                      slam_pose_result* results);

/* ------------------------------------------------------------------ stereo matching
 * Frame::ComputeStereoMatches (Frame.h:112, Frame.cc:794-964) for rectified stereo pairs
 * extracted by two extractor handles (left, right; same ORB parameters and image size):
 * row-band ORB matching (best Hamming < (TH_HIGH+TH_LOW)/2), 11x11 SAD search over +-5
 * columns on the pyramid level the handles hold, parabola sub-pixel fit, disparity gate,
 * median outlier cut.  mvuRight / mvDepth come back per left keypoint, -1 where unmatched. */
typedef struct slam_stereo slam_stereo;

slam_status slamhot_stereo_create(int device, slam_stereo** out);
void slamhot_stereo_destroy(slam_stereo* st);

/* Frame f of the last batch of `left` pairs with frame f of the last batch of `right`
 * (f < nframes).  Device inputs at cap stride per frame as produced by
 * slamhot_extract_batch_device: keypoints (slam_keypoint), descriptors (32 B), counts
 * (int32).  mbf, mb: Frame::mbf, Frame::mb.  Device outputs (float, cap per frame):
 * d_uright = mvuRight, d_depth = mvDepth; optional d_sad (int32, cap per frame, may be NULL):
 * the SAD of each kept match before the median cut, -1 otherwise.  Asynchronous on hip_stream
 * (NULL = the handle's stream); both extractors' work must be complete or ordered before it. */
slam_status slamhot_stereo_match_batch_device(slam_stereo* st, slam_extractor* left, slam_extractor* right,
                                              int nframes, const void* d_kps_left, const void* d_desc_left,
                                              const void* d_n_left, const void* d_kps_right,
                                              const void* d_desc_right, const void* d_n_right, int cap,
                                              float mbf, float mb, void* d_uright, void* d_depth, void* d_sad,
                                              void* hip_stream);

/* void Frame::ComputeStereoMatches() (Frame.cc:794-964) for one stereo Frame whose two images
 * were just extracted by `left` and `right` (slamhot_extract on each: their pyramids are still on
 * the device) — the host-buffer form the Frame constructor calls: the keypoints / descriptors
 * the two extractions returned in, mvuRight / mvDepth (n_left each, -1 where unmatched) out. */
slam_status slamhot_compute_stereo_matches(slam_stereo* st, slam_extractor* left, slam_extractor* right, int n_left,
                                           const slam_keypoint* kps_left, const uint8_t* desc_left, int n_right,
                                           const slam_keypoint* kps_right, const uint8_t* desc_right, float mbf,
                                           float mb, float* uright, float* depth);

/* ------------------------------------------------------------------ LocalMapping matchers
 * The Hamming-heavy work LocalMapping runs around local BA. */
typedef struct slam_mapper slam_mapper;

slam_status slamhot_mapper_create(int device, slam_mapper** out);
void slamhot_mapper_destroy(slam_mapper* mp);

/* void MapPoint::ComputeDistinctiveDescriptors() (MapPoint.h, MapPoint.cc:349-423) for n_mp
 * MapPoints at once.  MapPoint i's observed descriptors — non-bad KeyFrames in observation-map
 * order, left then right index per KeyFrame, exactly the reference's vDescriptors — are
 * desc[off[i] .. off[i+1]) (32 B each).  best[i] = the index, relative to off[i], of the
 * descriptor with the least median distance to the others (vDists[0.5*(N-1)], first on ties),
 * -1 when MapPoint i has none (mDescriptor unchanged). */
slam_status slamhot_distinctive_descriptors(slam_mapper* mp, int n_mp, const int32_t* off, const uint8_t* desc,
                                            int32_t* best);

/* A KeyFrame as SearchForTriangulation_ reads it (pinhole, NLeft == -1). */
typedef struct slam_tri_kf {
    int32_t n;
    const slam_keypoint* kps_un;  /* mvKeysUn (pt, octave, angle) */
    const float* uright;          /* mvuRight (NULL = all -1) */
    const uint8_t* desc;          /* mDescriptors, n x 32 */
    const uint8_t* has_mp;        /* GetMapPoint(i) != NULL */
    int32_t n_nodes;              /* mFeatVec as CSR: node ids ascending, their feature lists */
    const int32_t* node_id;       /* n_nodes */
    const int32_t* node_off;      /* n_nodes + 1 */
    const int32_t* node_feat;     /* node_off[n_nodes] feature indices */
    int32_t nlevels;
    const float* scale;           /* mvScaleFactors */
    const float* level_sigma2;    /* mvLevelSigma2 */
    float Rcw[9], tcw[3];         /* GetRotation_() / GetTranslation_() (Tcw_, KeyFrame.cc:1076-1084) */
    float Ow[3];                  /* GetCameraCenter_() (Ow_, KeyFrame.cc:1086-1089) */
    float cam[4];                 /* mpCamera parameters fx, fy, cx, cy (Pinhole::toK_) */
} slam_tri_kf;

/* One SearchForTriangulation_ call: KeyFrames kfs[kf1], kfs[kf2].  The epipole, R12, t12 and
 * the F12 that Pinhole::epipolarConstrain_ rebuilds from them on every call are computed on
 * the device from the two KeyFrames' poses and cameras with the reference binary's arithmetic
 * (ORBmatcher.cc:1215-1240, Pinhole.cpp:159-181).  The cv::Matx33f F12 argument
 * of the reference is not read on this (pinhole) path, so it has no field here. */
typedef struct slam_tri_pair {
    int32_t kf1, kf2;
    uint8_t only_stereo, coarse, pad[2];
} slam_tri_pair;

/* int ORBmatcher::SearchForTriangulation_(KeyFrame* pKF1, KeyFrame* pKF2, cv::Matx33f F12,
 * vector<pair<size_t,size_t>>& vMatchedPairs, bool bOnlyStereo, bool bCoarse)
 * (ORBmatcher.h, ORBmatcher.cc:1208-1433) for n_pairs pairs in one launch (LocalMapping::
 * CreateNewMapPoints calls it for every neighbour of the new KeyFrame, LocalMapping.cc:485).
 * check_ori = the matcher's mbCheckOrientation.  Outputs: match12[p * cap + idx1] = idx2 or -1
 * (cap >= kfs[pairs[p].kf1].n; vMatchedPairs = the idx1-ordered non-negative entries),
 * nmatches[p]. */
slam_status slamhot_search_for_triangulation(slam_mapper* mp, int n_kfs, const slam_tri_kf* kfs, int n_pairs,
                                             const slam_tri_pair* pairs, int check_ori, int cap,
                                             int32_t* match12, int32_t* nmatches);

/* int ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, float th, bool bRight)
 * (ORBmatcher.cc:1629-1818, bRight = false, NLeft == -1), search half: for every MapPoint the
 * projection into pKF, distance / viewing-angle gates, PredictScale, GetFeaturesInArea and the
 * chi2-gated best descriptor (first least distance in the reference's candidate order).
 * KF: the KeyFrame as a frame view (kps_un, uright, desc, grid bounds, Tcw, camera, level
 * tables; mp_state unused); inv_level_sigma2 = mvInvLevelSigma2.  mps: pos / normal / distances /
 * is_bad, seen = IsInKeyFrame(pKF).  Outputs: best_idx[i] (-1 = skipped or no candidate),
 * best_dist[i] (256 = none).  MapPoint i fuses iff best_dist[i] <= TH_LOW (50), applied in list
 * order by the caller (Replace / AddObservation, :1789-1812) — the search never depends on those
 * updates: they change only the skip flags (isBad, IsInKeyFrame), which the caller re-checks, and
 * the descriptors of MapPoints already processed or already in pKF. */
slam_status slamhot_fuse_search(slam_mapper* mp, const slam_frame_view* KF, const float* inv_level_sigma2,
                                int n_mp, const slam_mp_geom* mps, const uint8_t* mp_desc, float th,
                                int32_t* best_idx, int32_t* best_dist);

/* ------------------------------------------------------------------ stereo rectification
 * cv::remap(im, imRect, M1, M2, cv::INTER_LINEAR) with the CV_32F maps of
 * cv::initUndistortRectifyMap (stereo_euroc.cc:117-118, 168-169), BORDER_CONSTANT 0, for
 * batches of frames on the device.  The maps are converted once at create time to the
 * fixed-point form remap uses internally (value * 32 rounded to nearest even, 5-bit fractions,
 * 2^15-scaled bilinear weights). */
typedef struct slam_rectifier slam_rectifier;

/* map_x / map_y: host float maps, dst_w x dst_h (row-major); sources are src_w x src_h. */
slam_status slamhot_rectifier_create(int device, int src_w, int src_h, int dst_w, int dst_h, const float* map_x,
                                     const float* map_y, slam_rectifier** out);
void slamhot_rectifier_destroy(slam_rectifier* r);

/* nframes source images (device, u8, row pitch src_pitch, frame stride src_stride bytes) to
 * nframes destination images (dst_w x dst_h, pitch dst_pitch, stride dst_stride).
 * Asynchronous on hip_stream (NULL = the handle's stream). */
slam_status slamhot_rectify_batch_device(slam_rectifier* r, int nframes, const void* d_src, int src_pitch,
                                         int64_t src_stride, void* d_dst, int dst_pitch, int64_t dst_stride,
                                         void* hip_stream);

/* ------------------------------------------------------------------ per-sequence tracking
 * The stereo tracking chain of Tracking::Track for rectified stereo (BASELINE.json configs[4]),
 * device-resident: per frame cv::remap x2 -> ORBextractor x2 -> Frame::ComputeStereoMatches ->
 * TrackWithMotionModel (SearchByProjection(F, LastFrame) + PoseOptimization) when a velocity
 * exists, else / on its failure ComputeBoW + SearchByBoW(reference KF, F) + PoseOptimization ->
 * SearchLocalPoints -> PoseOptimization -> NeedNewKeyFrame / CreateNewKeyFrame
 * (Tracking.cc:1256-3330), with every
 * decision taken on the device.  nseq sequences advance in lock-step (one frame each per step);
 * the map is the reference KeyFrame of each sequence (DESIGN.md §4g states what LocalMapping-side
 * bookkeeping is left out). */
typedef struct slam_tracker slam_tracker;

typedef struct slam_tracker_config {
    int32_t nseq, width, height;
    slam_orb_params orb;          /* both extractors (EuRoC: 1200, 1.2, 8, 20, 7) */
    slam_camera cam;              /* rectified Camera.fx, fy, cx, cy, bf */
    float th_depth;               /* ThDepth in baselines (35): mThDepth = bf * ThDepth / fx */
    const float* map_lx;          /* initUndistortRectifyMap maps (width x height, float), or NULL */
    const float* map_ly;          /* when the inputs are already rectified */
    const float* map_rx;
    const float* map_ry;
} slam_tracker_config;

typedef struct slam_track_record {   /* one step of one sequence */
    float Tcw[16];                   /* mCurrentFrame.mTcw after the step */
    int32_t n, n_stereo;             /* N, features with mvDepth > 0 */
    int32_t n_bow;                   /* SearchByBoW(mpReferenceKF, F) */
    int32_t n_inl_ref;               /* TrackReferenceKeyFrame's nmatchesMap */
    int32_t n_local;                 /* SearchByProjection matches of SearchLocalPoints */
    int32_t n_inl;                   /* TrackLocalMap's mnMatchesInliers */
    int32_t is_keyframe, lost, initialized;
    int32_t n_motion;                /* TrackWithMotionModel's SearchByProjection(F, LastFrame) matches
                                        (after the 2 th retry; 0 = not tried: no velocity) */
    int32_t motion;                  /* 1: the first pose came from the motion model (n_bow = 0, the
                                        reference never ran TrackReferenceKeyFrame) */
    int32_t status;                  /* 0 ok; 1 a SearchByProjection candidate overflow voided the step:
                                        the sequence kept its previous state (lost = 1) */
} slam_track_record;

typedef struct slam_track_state {    /* a sequence's tracking state between steps (read back) */
    float V[16];                     /* mVelocity, valid when has_vel */
    float Tlr[16];                   /* mlRelativeFramePoses.back(): last frame w.r.t. its reference KF */
    float Tref[16];                  /* the reference KeyFrame's pose */
    int32_t has_vel, nkf;            /* KeyFrames created in the sequence (KeyFramesInMap) */
    int32_t last_n, cap;             /* mLastFrame.N; cap: capacity of the arrays below (in) */
    slam_keypoint* last_kps;         /* mLastFrame.mvKeysUn */
    int32_t* last_mp;                /* mLastFrame.mvpMapPoints as reference-KeyFrame MapPoint slots, -1 = NULL */
} slam_track_state;

typedef struct slam_track_frame {    /* the last step's per-feature results of one sequence */
    int32_t n, cap;                  /* N; cap: capacity of the arrays (in) */
    float* uright;                   /* mvuRight (ComputeStereoMatches) */
    int32_t* bow_match;              /* SearchByBoW(refKF, F): the KF feature (= MapPoint slot) per feature */
    int32_t* motion_match;           /* SearchByProjection(F, LastFrame): MapPoint slot per feature */
    int32_t* local_match;            /* SearchLocalPoints' SearchByProjection: MapPoint slot per feature */
    int32_t* mappoints;              /* mvpMapPoints at the end of the step (outliers removed) */
} slam_track_frame;

typedef struct slam_track_keyframe { /* the reference KeyFrame of one sequence (read back) */
    float Tcw[16];                   /* the sequence's current pose */
    int32_t initialized, n_ref, n, cap;  /* cap: capacity of the arrays below (in) */
    slam_keypoint* kps;
    uint8_t* desc;                   /* n x 32 */
    uint8_t* mp_valid;
    float* mp_pos;                   /* n x 3 */
    float* mp_normal;                /* n x 3 */
    float* mp_min_dist;
    float* mp_max_dist;
    uint8_t* mp_desc;                /* n x 32 */
} slam_track_keyframe;

/* voc stays owned by the caller and must outlive the tracker. */
slam_status slamhot_tracker_create(int device, const slam_tracker_config* cfg, slam_vocab* voc, slam_tracker** out);
void slamhot_tracker_destroy(slam_tracker* t);
/* One frame of every sequence: nseq left and nseq right u8 images in device memory (raw when the
 * tracker holds rectification maps).  Asynchronous: nothing waits on the host. */
slam_status slamhot_tracker_step_device(slam_tracker* t, const void* d_left, int left_pitch, int64_t left_stride,
                                        const void* d_right, int right_pitch, int64_t right_stride);
/* The last step's records (nseq), synchronising; SLAM_ECAP if a sequence's SearchByProjection
 * candidates overflowed (its matches would be incomplete). */
slam_status slamhot_tracker_records(slam_tracker* t, slam_track_record* out);
slam_status slamhot_tracker_keyframe(slam_tracker* t, int seq, slam_track_keyframe* kf);
/* The motion-model state and last frame of sequence seq (synchronising). */
slam_status slamhot_tracker_state(slam_tracker* t, int seq, slam_track_state* st);
/* The last step's per-feature match arrays of sequence seq (synchronising; NULL arrays skipped). */
slam_status slamhot_tracker_frame(slam_tracker* t, int seq, slam_track_frame* fr);

#ifdef __cplusplus
}
#endif
#endif /* SLAMHOT_H */
