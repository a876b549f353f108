/*
 * MAM3SLAM::Settings — the part of the reference's settings reader (include/Settings.h, src/Settings.cc) the hot path
 * is built from: File.version (Agent.cc:22-29 requires "1.0"), Camera.type and Camera1.* (readCamera1, Settings.cc:
 * 184-270: Pinhole with optional k1 k2 p1 p2 [k3] distortion, KannalaBrandt8 with k1..k4), Camera.width / height /
 * fps, and the five ORB keys (readORB, Settings.cc:443-451: ORBextractor.nFeatures, scaleFactor, nLevels, iniThFAST,
 * minThFAST). The file is the reference's OpenCV FileStorage YAML (%YAML:1.0, flat "key: value" lines, '#'
 * comments); reals are read as double and narrowed to float as readParameter<float> does, integers as int. A missing
 * required key throws std::runtime_error (the reference prints it and exits).
 */
#ifndef MAM3SLAM_SETTINGS_H
#define MAM3SLAM_SETTINGS_H

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "ORBextractor.h"
#include "Types.h"

namespace MAM3SLAM {

class Settings {
public:
    enum CameraType { PinHole = 0, Rectified = 1, KannalaBrandt = 2 };   // Settings.h:38-42

    explicit Settings(const std::string& configFile);

    CameraType cameraType() const { return cameraType_; }
    const GeometricCamera& camera1() const { return camera1_; }
    /* Pinhole distortion k1 k2 p1 p2 [k3] (empty for KannalaBrandt8, whose k1..k4 are in the camera) */
    const std::vector<float>& camera1DistortionCoef() const { return vPinHoleDistorsion1_; }
    int imageWidth() const { return width_; }
    int imageHeight() const { return height_; }
    float fps() const { return fps_; }

    int nFeatures() const { return nFeatures_; }
    float scaleFactor() const { return scaleFactor_; }
    int nLevels() const { return nLevels_; }
    int initThFAST() const { return initThFAST_; }
    int minThFAST() const { return minThFAST_; }

    /* Tracking's extractor (Tracking.cc:600-606): new ORBextractor(nFeatures, scaleFactor, nLevels, iniThFAST,
     * minThFAST) on `device` */
    std::unique_ptr<ORBextractor> makeORBextractor(int device = 0) const;

    /* every "key: value" of the file (values as written, quotes removed) */
    const std::map<std::string, std::string>& values() const { return kv_; }

private:
    std::map<std::string, std::string> kv_;
    CameraType cameraType_ = PinHole;
    GeometricCamera camera1_;
    std::vector<float> vPinHoleDistorsion1_;
    int width_ = 0, height_ = 0;
    float fps_ = 0.f;
    int nFeatures_ = 0, nLevels_ = 0, initThFAST_ = 0, minThFAST_ = 0;
    float scaleFactor_ = 0.f;

    bool has(const std::string& k) const { return kv_.count(k) != 0; }
    float readFloat(const std::string& k, bool required = true) const;
    int readInt(const std::string& k, bool required = true) const;
    std::string readString(const std::string& k, bool required = true) const;
};

}  // namespace MAM3SLAM
#endif
