// MAM3SLAM::ORBextractor over the gfx950 extractor (include/mam3slam/ORBextractor.h).
// Reference: include/ORBextractor.h:43-100, src/ORBextractor.cc:409-469 (tables), :1086-1168 (operator()).
#include <cstring>
#include <stdexcept>
#include <string>

#include "mam3slam/ORBextractor.h"

namespace MAM3SLAM {

static void throwOn(int rc, const char* what) {
    if (rc < 0) throw std::runtime_error(std::string(what) + " failed (" + std::to_string(rc) + "): " + mam_last_error());
}

ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST,
                           int device)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST) {
    mam_orb_params p;
    p.nfeatures = _nfeatures;
    p.scale_factor = _scaleFactor;
    p.nlevels = _nlevels;
    p.ini_th_fast = _iniThFAST;
    p.min_th_fast = _minThFAST;
    p.fp_policy = 0;   // the reference binary's arithmetic (mam_orb.h)
    throwOn(mam_orb_create(&p, device, &ctx), "mam_orb_create");
    std::vector<float> s(4 * (size_t)nlevels);
    mnFeaturesPerLevel.resize(nlevels);
    throwOn(mam_orb_scales(ctx, s.data()), "mam_orb_scales");
    throwOn(mam_orb_features_per_level(ctx, mnFeaturesPerLevel.data()), "mam_orb_features_per_level");
    mvScaleFactor.assign(s.begin(), s.begin() + nlevels);
    mvInvScaleFactor.assign(s.begin() + nlevels, s.begin() + 2 * nlevels);
    mvLevelSigma2.assign(s.begin() + 2 * nlevels, s.begin() + 3 * nlevels);
    mvInvLevelSigma2.assign(s.begin() + 3 * nlevels, s.begin() + 4 * nlevels);
    capacity = mam_orb_max_keypoints(ctx);
    throwOn(capacity, "mam_orb_max_keypoints");
    kbuf.resize(capacity);
}

ORBextractor::~ORBextractor() {
    if (ctx) mam_orb_destroy(ctx);
}

int ORBextractor::operator()(const ImageView& image, const ImageView& /*mask*/, std::vector<KeyPoint>& keypoints,
                             Mat8U& descriptors, std::vector<int>& vLappingArea) {
    if (image.empty()) return -1;   // ORBextractor.cc:1090-1091
    if (vLappingArea.size() < 2) throw std::invalid_argument("vLappingArea needs two entries");
    descriptors.create(capacity, 32);
    int n = 0, mono = 0;
    const int rc = mam_orb_extract(ctx, image.data, image.cols, image.rows, image.step, vLappingArea[0],
                                   vLappingArea[1], kbuf.data(), descriptors.data.data(), capacity, &n, &mono);
    throwOn(rc, "mam_orb_extract");
    keypoints.resize(n);
    if (n) std::memcpy(keypoints.data(), kbuf.data(), sizeof(KeyPoint) * (size_t)n);
    descriptors.rows = n;
    descriptors.data.resize((size_t)n * 32);
    return mono;
}

std::vector<Mat8U> ORBextractor::GetImagePyramid() const {
    std::vector<Mat8U> out(nlevels);
    for (int l = 0; l < nlevels; l++) {
        int w = 0, h = 0;
        throwOn(mam_orb_get_level(ctx, 0, l, nullptr, &w, &h), "mam_orb_get_level(size)");
        out[l].create(h, w);
        throwOn(mam_orb_get_level(ctx, 0, l, out[l].data.data(), &w, &h), "mam_orb_get_level");
    }
    return out;
}

}  // namespace MAM3SLAM
