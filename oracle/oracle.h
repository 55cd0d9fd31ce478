/*
 * oracle.h — CPU restatement of the ORB-SLAM3 hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline.  The product (libslamhot.so) never
 * links or calls it.
 *
 * PARITY STATUS: "parity unpinned" against the real reference.  The reference path
 * cannot be built here (no OpenCV, no Eigen: SURVEY.md §8c) and ships no golden
 * vectors for this path.  Each function restates the reference code cited next to it;
 * the OpenCV 4.2.0 primitives it calls (FAST, resize, GaussianBlur, fastAtan2) are
 * restated from the published OpenCV 4.2.0 algorithm, and glibc
 * sincosf is used directly (the device restatement is checked bit-exact against it over
 * every float in [0, 2*pi)).  Known-answer tests pin the restated primitives.
 */
#ifndef SLAMHOT_ORACLE_H
#define SLAMHOT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/slamhot.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ORBextractor::operator() restated (ORBextractor.cc:1068-1150). */
int oracle_extract(const slam_orb_params* p, const uint8_t* img, int w, int h, size_t stride,
                   int lap0, int lap1, slam_keypoint* kps, uint8_t* desc, int cap, int* n,
                   int* mono_index);

/* Scale tables (ORBextractor.cc:408-444). */
void oracle_levels(const slam_orb_params* p, float* scale, float* inv_scale, float* sigma2,
                   float* inv_sigma2, int32_t* nfeat);

/* Pyramid (ORBextractor.cc:1152-1177): writes level l into out + offsets[l] (tight rows). */
int oracle_pyramid(const slam_orb_params* p, const uint8_t* img, int w, int h, size_t stride,
                   uint8_t* out, size_t out_cap, int* lw, int* lh, size_t* offsets);

/* cv::resize(INTER_LINEAR) for 8U, one channel (OpenCV 4.2.0 resizeGeneric_ fixed point). */
void oracle_resize_linear(const uint8_t* src, int sw, int sh, size_t sstep, uint8_t* dst,
                          int dw, int dh, size_t dstep);

/* cv::FAST(img, kps, threshold, nonmax=true) on one ROI (OpenCV 4.2.0 FAST_t<16>).
 * Writes x, y, score triples; returns the count (or -needed if cap too small). */
int oracle_fast(const uint8_t* roi, int w, int h, size_t stride, int threshold, int32_t* xys,
                int cap);

/* GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) 8U fixed point.  ed_kernel=1 selects the
 * error-diffused Q8 kernel [18,34,48,56,48,34,18]; 0 the per-tap rounded one. */
void oracle_gaussian_blur7(const uint8_t* src, int w, int h, size_t sstep, uint8_t* dst,
                           size_t dstep, int ed_kernel);

/* cv::fastAtan2 (OpenCV 4.2.0 atan_f32) and glibc sincosf. */
float oracle_fast_atan2(float y, float x);
void oracle_sincosf(float x, float* s, float* c);

/* Per-level keypoints before descriptors: ComputeKeyPointsOctTree (ORBextractor.cc:763-878).
 * Writes keypoints of every level in level order; counts[l] per level. */
int oracle_keypoints_octree(const slam_orb_params* p, const uint8_t* img, int w, int h,
                            size_t stride, slam_keypoint* kps, int cap, int32_t* counts);

/* Hamming distance (ORBmatcher.cc:2561-2577). */
int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* CPU baseline: extract nframes images with nthreads std::threads (one frame per
 * thread at a time, like Frame.cc:119-122).  Returns total keypoints. */
long oracle_extract_many(const slam_orb_params* p, int nframes, const uint8_t* imgs, int w,
                         int h, size_t stride, int lap0, int lap1, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
