/*
 * rectify_oracle.cpp — CPU restatement of cv::remap(src, dst, map1, map2, INTER_LINEAR)
 * with CV_32FC1 maps and the default BORDER_CONSTANT / 0, as stereo_euroc.cc:168-169 calls it
 * [OpenCV 4.2.0, imgproc/src/imgwarp.cpp: RemapInvoker + remapBilinear<FixedPtCast<int,
 * uchar, 15>>]: each map value is scaled by INTER_TAB_SIZE = 32 and rounded to nearest even
 * (saturate_cast<int>), split into integer part (>> 5) and a 5+5-bit fraction; the 2x2 tap
 * weights are the fixed-point products (32-fx)(32-fy) ... scaled to 2^15 (exact: no
 * correction step applies to INTER_LINEAR), result (sum + 2^14) >> 15.  Taps outside the
 * source read the border value 0; a pixel whose whole 2x2 neighbourhood is outside is 0.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Parity unpinned (OpenCV is not in this image).
 */
#include <cmath>
#include <cstdint>
#include <cstring>

extern "C" {

void oracle_remap_linear(const uint8_t* src, int sw, int sh, int spitch, const float* map_x, const float* map_y,
                         int dw, int dh, uint8_t* dst, int dpitch) {
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            const float mx = map_x[(size_t)y * dw + x], my = map_y[(size_t)y * dw + x];
            // saturate_cast<int>(v * INTER_TAB_SIZE): round to nearest even, saturating
            const float fxs = mx * 32.0f, fys = my * 32.0f;
            const double cx = std::nearbyint((double)fxs), cy = std::nearbyint((double)fys);
            const int X = cx >= 2147483647.0 ? 2147483647 : cx <= -2147483648.0 ? (int)-2147483648LL : (int)cx;
            const int Y = cy >= 2147483647.0 ? 2147483647 : cy <= -2147483648.0 ? (int)-2147483648LL : (int)cy;
            // saturate_cast<short>(X >> INTER_BITS)
            int sx = X >> 5, sy = Y >> 5;
            sx = sx < -32768 ? -32768 : sx > 32767 ? 32767 : sx;
            sy = sy < -32768 ? -32768 : sy > 32767 ? 32767 : sy;
            const int fx = X & 31, fy = Y & 31;
            const int w00 = (32 - fx) * (32 - fy) * 32, w01 = fx * (32 - fy) * 32;
            const int w10 = (32 - fx) * fy * 32, w11 = fx * fy * 32;
            uint8_t out;
            if ((unsigned)sx < (unsigned)(sw - 1) && (unsigned)sy < (unsigned)(sh - 1)) {
                const uint8_t* S = src + (size_t)sy * spitch + sx;
                const int v = S[0] * w00 + S[1] * w01 + S[spitch] * w10 + S[spitch + 1] * w11;
                out = (uint8_t)((v + (1 << 14)) >> 15);
            } else if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) {
                out = 0;
            } else {
                auto at = [&](int yy, int xx) -> int {
                    return (xx >= 0 && xx < sw && yy >= 0 && yy < sh) ? src[(size_t)yy * spitch + xx] : 0;
                };
                const int v = at(sy, sx) * w00 + at(sy, sx + 1) * w01 + at(sy + 1, sx) * w10 + at(sy + 1, sx + 1) * w11;
                int r = (v + (1 << 14)) >> 15;
                out = (uint8_t)(r < 0 ? 0 : r > 255 ? 255 : r);
            }
            dst[(size_t)y * dpitch + x] = out;
        }
}

}  // extern "C"
