/*
 * MAM3SLAM::ORBextractor — the reference class (include/ORBextractor.h:43-100) over the gfx950 extractor
 * (C-ABI include/mam_orb.h). Same constructor arguments, same operator() contract (returns monoIndex, -1 on an
 * empty image; keypoints in the lapping placement order of src/ORBextractor.cc:1123-1165; descriptors N x 32),
 * same getters. Differences: OpenCV types are replaced by Types.h equivalents, and the image pyramid is a
 * device-resident object copied to the host on demand (GetImagePyramid) instead of a public member that every
 * call refills.
 *
 * Not thread-safe, like the reference: one instance per tracking thread.
 */
#ifndef MAM3SLAM_ORBEXTRACTOR_H
#define MAM3SLAM_ORBEXTRACTOR_H

#include <vector>

#include "Types.h"

namespace MAM3SLAM {

class ORBextractor {
public:
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device = 0);
    ~ORBextractor();
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    /* ORBextractor.cc:1086-1168. mask is ignored, as in the reference. Throws std::runtime_error on device
     * errors (the reference has no error path besides the empty image). */
    int operator()(const ImageView& image, const ImageView& mask, std::vector<KeyPoint>& keypoints,
                   Mat8U& descriptors, std::vector<int>& vLappingArea);

    int inline GetLevels() const { return nlevels; }
    float inline GetScaleFactor() const { return (float)scaleFactor; }
    std::vector<float> inline GetScaleFactors() const { return mvScaleFactor; }
    std::vector<float> inline GetInverseScaleFactors() const { return mvInvScaleFactor; }
    std::vector<float> inline GetScaleSigmaSquares() const { return mvLevelSigma2; }
    std::vector<float> inline GetInverseScaleSigmaSquares() const { return mvInvLevelSigma2; }
    std::vector<int> inline GetFeaturesPerLevel() const { return mnFeaturesPerLevel; }

    /* mvImagePyramid of the last call (levels without the 19-px border). */
    std::vector<Mat8U> GetImagePyramid() const;

    mam_orb_ctx* handle() const { return ctx; }

protected:
    int nfeatures;
    double scaleFactor;
    int nlevels;
    int iniThFAST;
    int minThFAST;
    std::vector<int> mnFeaturesPerLevel;
    std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;

private:
    mam_orb_ctx* ctx = nullptr;
    int capacity = 0;
    std::vector<mam_keypoint> kbuf;
};

}  // namespace MAM3SLAM
#endif
