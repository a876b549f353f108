// orb_simd.cpp — TEST INFRASTRUCTURE ONLY (the CPU baseline's second column; see orb_oracle.h).
//
// AVX2 restatements of the three image primitives the reference's ORBextractor gets from OpenCV's SIMD code paths
// (OpenCV 4.5.4 is not vendored in the reference; the algorithms are the published ones):
//   resize INTER_LINEAR 8U   imgproc/resize.cpp VResizeLinearVec_32s8u (the vertical pass: >> 4 to int16,
//                            mulhi by the int16 betas, saturating adds, + 2, >> 2, saturating pack), HResizeLinear
//                            left as the scalar integer pass
//   GaussianBlur 7x7         the fixed-point separable filter (ufixedpoint16 rows, ufixedpoint32 columns,
//                            round-half-up >> 16) over 16 / 8 pixels per instruction, reflect-101 borders scalar
//   FAST TYPE_9_16           features2d/fast.cpp's universal-intrinsics path: per 32 pixels the quick 4-point test,
//                            then the run length of consecutive brighter / darker circle pixels over the 25-entry
//                            circle by saturating byte counters; the corners' scores and the non-max suppression
//                            are the scalar code's
// Every output byte / keypoint equals the scalar oracle's (tests/test_oracle_kat.py compares them); the baseline
// times the extractor with these (bench.py cpu_baseline: "extract_simd").
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

namespace oracle_simd {

inline uint8_t satU8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }
inline int16_t sat16(int v) { return (int16_t)(v < -32768 ? -32768 : v > 32767 ? 32767 : v); }

// ---- resize: the vertical pass of columns x < xvec with the SIMD formula, 16 at a time
void resize_vline(const int* r0, const int* r1, int b0, int b1, int xvec, int dw, uint8_t* D) {
    const __m256i vb0 = _mm256_set1_epi16((int16_t)b0), vb1 = _mm256_set1_epi16((int16_t)b1);
    const __m256i two = _mm256_set1_epi16(2);
    int x = 0;
    for (; x + 16 <= xvec; x += 16) {
        const __m256i a0 = _mm256_srai_epi32(_mm256_loadu_si256((const __m256i*)(r0 + x)), 4);
        const __m256i a1 = _mm256_srai_epi32(_mm256_loadu_si256((const __m256i*)(r0 + x + 8)), 4);
        const __m256i c0 = _mm256_srai_epi32(_mm256_loadu_si256((const __m256i*)(r1 + x)), 4);
        const __m256i c1 = _mm256_srai_epi32(_mm256_loadu_si256((const __m256i*)(r1 + x + 8)), 4);
        // packs works per 128-bit lane: restore element order
        const __m256i h0 = _mm256_permute4x64_epi64(_mm256_packs_epi32(a0, a1), 0xD8);
        const __m256i h1 = _mm256_permute4x64_epi64(_mm256_packs_epi32(c0, c1), 0xD8);
        const __m256i s = _mm256_adds_epi16(_mm256_mulhi_epi16(h0, vb0), _mm256_mulhi_epi16(h1, vb1));
        const __m256i r = _mm256_srai_epi16(_mm256_adds_epi16(s, two), 2);
        const __m256i p = _mm256_permute4x64_epi64(_mm256_packus_epi16(r, r), 0xD8);
        _mm_storeu_si128((__m128i*)(D + x), _mm256_castsi256_si128(p));
    }
    for (; x < xvec; x++) {
        const int16_t h0 = sat16(r0[x] >> 4), h1 = sat16(r1[x] >> 4);
        const int16_t m0 = (int16_t)(((int)h0 * b0) >> 16), m1 = (int16_t)(((int)h1 * b1) >> 16);
        const int16_t s = sat16((int)m0 + (int)m1);
        const int16_t r = sat16((int)s + 2);
        D[x] = satU8(r >> 2);
    }
    for (; x < dw; x++) D[x] = satU8((r0[x] * b0 + r1[x] * b1 + (1 << 21)) >> 22);
}

// ---- GaussianBlur 7x7 fixed point
static const int kTaps[7] = {18, 34, 48, 56, 48, 34, 18};

inline int refl101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

void gaussian7(const uint8_t* src, int w, int h, size_t sstride, uint8_t* dst, size_t dstride) {
    // the row pass in uint16 (sum of the taps = 256: at most 255 * 256 = 65280)
    std::vector<uint16_t> hb((size_t)w * h + 16);
    __m256i tap[7];
    for (int i = 0; i < 7; i++) tap[i] = _mm256_set1_epi16((int16_t)kTaps[i]);
    for (int y = 0; y < h; y++) {
        const uint8_t* s = src + (size_t)y * sstride;
        uint16_t* o = hb.data() + (size_t)y * w;
        int x = 0;
        auto scalar = [&](int xx) {
            uint32_t acc = 0;
            for (int i = -3; i <= 3; i++) acc += (uint32_t)kTaps[i + 3] * s[refl101(xx + i, w)];
            o[xx] = (uint16_t)acc;
        };
        for (; x < std::min(3, w); x++) scalar(x);
        for (; x + 16 <= w - 3; x += 16) {
            __m256i acc = _mm256_setzero_si256();
            for (int i = 0; i < 7; i++) {
                const __m256i v = _mm256_cvtepu8_epi16(_mm_loadu_si128((const __m128i*)(s + x + i - 3)));
                acc = _mm256_add_epi16(acc, _mm256_mullo_epi16(v, tap[i]));
            }
            _mm256_storeu_si256((__m256i*)(o + x), acc);
        }
        for (; x < w; x++) scalar(x);
    }
    // the column pass in uint32, 8 pixels per step
    __m256i tap32[7];
    for (int i = 0; i < 7; i++) tap32[i] = _mm256_set1_epi32(kTaps[i]);
    const __m256i half = _mm256_set1_epi32(32768), c255 = _mm256_set1_epi32(255);
    for (int y = 0; y < h; y++) {
        const uint16_t* rows[7];
        for (int j = 0; j < 7; j++) rows[j] = hb.data() + (size_t)refl101(y + j - 3, h) * w;
        uint8_t* o = dst + (size_t)y * dstride;
        int x = 0;
        for (; x + 8 <= w; x += 8) {
            __m256i acc = _mm256_setzero_si256();
            for (int j = 0; j < 7; j++) {
                const __m256i v = _mm256_cvtepu16_epi32(_mm_loadu_si128((const __m128i*)(rows[j] + x)));
                acc = _mm256_add_epi32(acc, _mm256_mullo_epi32(v, tap32[j]));
            }
            __m256i r = _mm256_min_epi32(_mm256_srli_epi32(_mm256_add_epi32(acc, half), 16), c255);
            const __m256i p16 = _mm256_packus_epi32(r, r);                 // lanes: [0..3 0..3 | 4..7 4..7]
            const __m256i p8 = _mm256_packus_epi16(p16, p16);
            const uint32_t lo = (uint32_t)_mm256_extract_epi32(p8, 0), hi = (uint32_t)_mm256_extract_epi32(p8, 4);
            memcpy(o + x, &lo, 4);
            memcpy(o + x + 4, &hi, 4);
        }
        for (; x < w; x++) {
            uint32_t s = 0;
            for (int j = 0; j < 7; j++) s += (uint32_t)kTaps[j] * rows[j][x];
            const uint32_t r = (s + 32768u) >> 16;
            o[x] = (uint8_t)(r > 255 ? 255 : r);
        }
    }
}

// ---- FAST 9/16
struct Kp {
    float x, y, response;
};

static void makeOffsets(int pixel[25], int rowStride) {
    static const int offsets16[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                                         {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};
    int k = 0;
    for (; k < 16; k++) pixel[k] = offsets16[k][0] + offsets16[k][1] * rowStride;
    for (; k < 25; k++) pixel[k] = pixel[k - 16];
}

static int cornerScore16(const uint8_t* ptr, const int pixel[], int threshold) {
    const int K = 8, N = K * 3 + 1;
    int k, v = ptr[0];
    short d[N];
    for (k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (k = 0; k < 16; k += 2) {
        int a = std::min((int)d[k + 1], (int)d[k + 2]);
        a = std::min(a, (int)d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, (int)d[k + 4]);
        a = std::min(a, (int)d[k + 5]);
        a = std::min(a, (int)d[k + 6]);
        a = std::min(a, (int)d[k + 7]);
        a = std::min(a, (int)d[k + 8]);
        a0 = std::max(a0, std::min(a, (int)d[k]));
        a0 = std::max(a0, std::min(a, (int)d[k + 9]));
    }
    int b0 = -a0;
    for (k = 0; k < 16; k += 2) {
        int b = std::max((int)d[k + 1], (int)d[k + 2]);
        b = std::max(b, (int)d[k + 3]);
        b = std::max(b, (int)d[k + 4]);
        b = std::max(b, (int)d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, (int)d[k + 6]);
        b = std::max(b, (int)d[k + 7]);
        b = std::max(b, (int)d[k + 8]);
        b0 = std::min(b0, std::max(b, (int)d[k]));
        b0 = std::min(b0, std::max(b, (int)d[k + 9]));
    }
    return -b0 - 1;
}

// x, y, response of the corners of the roi after non-max suppression, in the scalar code's order
void fast16(const uint8_t* img, int cols, int rows, size_t step, int threshold, std::vector<Kp>& keypoints) {
    const int K = 8, N = 16 + K + 1;
    int i, j, k, pixel[25];
    makeOffsets(pixel, (int)step);
    keypoints.clear();
    threshold = std::min(std::max(threshold, 0), 255);
    uint8_t threshold_tab[512];
    for (i = -255; i <= 255; i++) threshold_tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    if (cols < 7 || rows < 7) return;
    std::vector<uint8_t> bufv(cols * 3, 0);
    std::vector<int> cpv((cols + 1) * 3, 0);
    uint8_t* buf[3] = {bufv.data(), bufv.data() + cols, bufv.data() + cols * 2};
    int* cpbuf[3] = {cpv.data(), cpv.data() + (cols + 1), cpv.data() + (cols + 1) * 2};
    const __m256i delta = _mm256_set1_epi8((char)0x80), t8 = _mm256_set1_epi8((char)threshold);
    const __m256i kK = _mm256_set1_epi8((char)K);
    for (i = 3; i < rows - 2; i++) {
        const uint8_t* ptr = img + (size_t)i * step + 3;
        uint8_t* curr = buf[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3] + 1;
        memset(curr, 0, cols);
        int ncorners = 0;
        if (i < rows - 3) {
            j = 3;
            for (; j < cols - 32 - 3; j += 32, ptr += 32) {
                const __m256i v = _mm256_loadu_si256((const __m256i*)ptr);
                // brighter than v + t / darker than v - t, in signed byte order (saturated: no false hits)
                const __m256i v0 = _mm256_xor_si256(_mm256_adds_epu8(v, t8), delta);
                const __m256i v1 = _mm256_xor_si256(_mm256_subs_epu8(v, t8), delta);
                const __m256i x0 = _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(ptr + pixel[0])), delta);
                const __m256i x1 = _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(ptr + pixel[4])), delta);
                const __m256i x2 = _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(ptr + pixel[8])), delta);
                const __m256i x3 = _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(ptr + pixel[12])), delta);
                __m256i m0 = _mm256_and_si256(_mm256_cmpgt_epi8(x0, v0), _mm256_cmpgt_epi8(x1, v0));
                __m256i m1 = _mm256_and_si256(_mm256_cmpgt_epi8(v1, x0), _mm256_cmpgt_epi8(v1, x1));
                m0 = _mm256_or_si256(m0, _mm256_and_si256(_mm256_cmpgt_epi8(x1, v0), _mm256_cmpgt_epi8(x2, v0)));
                m1 = _mm256_or_si256(m1, _mm256_and_si256(_mm256_cmpgt_epi8(v1, x1), _mm256_cmpgt_epi8(v1, x2)));
                m0 = _mm256_or_si256(m0, _mm256_and_si256(_mm256_cmpgt_epi8(x2, v0), _mm256_cmpgt_epi8(x3, v0)));
                m1 = _mm256_or_si256(m1, _mm256_and_si256(_mm256_cmpgt_epi8(v1, x2), _mm256_cmpgt_epi8(v1, x3)));
                m0 = _mm256_or_si256(m0, _mm256_and_si256(_mm256_cmpgt_epi8(x3, v0), _mm256_cmpgt_epi8(x0, v0)));
                m1 = _mm256_or_si256(m1, _mm256_and_si256(_mm256_cmpgt_epi8(v1, x3), _mm256_cmpgt_epi8(v1, x0)));
                m0 = _mm256_or_si256(m0, m1);
                if (_mm256_testz_si256(m0, m0)) continue;
                __m256i c0 = _mm256_setzero_si256(), c1 = c0, max0 = c0, max1 = c0;
                for (k = 0; k < N; k++) {
                    const __m256i x = _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(ptr + pixel[k])), delta);
                    const __m256i b = _mm256_cmpgt_epi8(x, v0), d = _mm256_cmpgt_epi8(v1, x);
                    c0 = _mm256_and_si256(_mm256_sub_epi8(c0, b), b);   // run length of consecutive hits
                    c1 = _mm256_and_si256(_mm256_sub_epi8(c1, d), d);
                    max0 = _mm256_max_epu8(max0, c0);
                    max1 = _mm256_max_epu8(max1, c1);
                }
                const __m256i mx = _mm256_max_epu8(max0, max1);
                uint32_t m = (uint32_t)_mm256_movemask_epi8(_mm256_cmpgt_epi8(mx, kK));
                while (m) {
                    const int b = __builtin_ctz(m);
                    m &= m - 1;
                    cornerpos[ncorners++] = j + b;
                    curr[j + b] = (uint8_t)cornerScore16(ptr + b, pixel, threshold);
                }
            }
            for (; j < cols - 3; j++, ptr++) {
                const int v = ptr[0];
                const uint8_t* tab = &threshold_tab[0] - v + 255;
                int d = tab[ptr[pixel[0]]] | tab[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= tab[ptr[pixel[2]]] | tab[ptr[pixel[10]]];
                d &= tab[ptr[pixel[4]]] | tab[ptr[pixel[12]]];
                d &= tab[ptr[pixel[6]]] | tab[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= tab[ptr[pixel[1]]] | tab[ptr[pixel[9]]];
                d &= tab[ptr[pixel[3]]] | tab[ptr[pixel[11]]];
                d &= tab[ptr[pixel[5]]] | tab[ptr[pixel[13]]];
                d &= tab[ptr[pixel[7]]] | tab[ptr[pixel[15]]];
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)cornerScore16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
                if (d & 2) {
                    int vt = v + threshold, count = 0;
                    for (k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)cornerScore16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = buf[(i - 4 + 3) % 3];
        const uint8_t* pprev = buf[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3] + 1;
        ncorners = cornerpos[-1];
        for (k = 0; k < ncorners; k++) {
            j = cornerpos[k];
            const int score = prev[j];
            if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] && score > pprev[j] &&
                score > pprev[j + 1] && score > curr[j - 1] && score > curr[j] && score > curr[j + 1])
                keypoints.push_back({(float)j, (float)(i - 1), (float)score});
        }
    }
}

}  // namespace oracle_simd
