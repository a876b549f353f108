// MAM3SLAM::Settings (include/mam3slam/Settings.h): the reference's settings keys for the extractor and camera 1,
// read from its OpenCV FileStorage YAML (src/Settings.cc:184-270, 443-451; src/Agent.cc:22-29).
#include "../../include/mam3slam/Settings.h"

#include <cerrno>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace MAM3SLAM {

namespace {

std::string trim(const std::string& s) {
    const size_t a = s.find_first_not_of(" \t\r");
    if (a == std::string::npos) return "";
    const size_t b = s.find_last_not_of(" \t\r");
    return s.substr(a, b - a + 1);
}

}  // namespace

Settings::Settings(const std::string& configFile) {
    std::ifstream in(configFile);
    if (!in) throw std::runtime_error("Settings: cannot open " + configFile);
    std::string line;
    bool first = true;
    while (std::getline(in, line)) {
        if (first) {
            first = false;
            if (trim(line).rfind("%YAML", 0) == 0) continue;   // FileStorage's %YAML:1.0 directive
        }
        // strip a comment (outside quotes)
        bool q = false;
        for (size_t i = 0; i < line.size(); i++) {
            if (line[i] == '"') q = !q;
            if (line[i] == '#' && !q) {
                line.resize(i);
                break;
            }
        }
        const std::string t = trim(line);
        if (t.empty() || t == "---") continue;
        const size_t c = t.find(':');
        if (c == std::string::npos) continue;
        const std::string key = trim(t.substr(0, c));
        std::string val = trim(t.substr(c + 1));
        if (val.size() >= 2 && val.front() == '"' && val.back() == '"') val = val.substr(1, val.size() - 2);
        if (!key.empty()) kv_[key] = val;
    }
    // Agent.cc:22-29: the settings file must declare File.version "1.0"
    if (readString("File.version", false) != "1.0")
        throw std::runtime_error("Settings: " + configFile + " is not a File.version \"1.0\" settings file");
    // readCamera1 (Settings.cc:184-270)
    const std::string model = readString("Camera.type");
    if (model == "PinHole" || model == "Rectified") {
        cameraType_ = model == "PinHole" ? PinHole : Rectified;
        camera1_ = Pinhole(readFloat("Camera1.fx"), readFloat("Camera1.fy"), readFloat("Camera1.cx"),
                           readFloat("Camera1.cy"));
        if (cameraType_ == PinHole && has("Camera1.k1")) {   // optional radial-tangential distortion
            vPinHoleDistorsion1_ = {readFloat("Camera1.k1"), readFloat("Camera1.k2"), readFloat("Camera1.p1"),
                                    readFloat("Camera1.p2")};
            if (has("Camera1.k3")) vPinHoleDistorsion1_.push_back(readFloat("Camera1.k3"));
        }
    } else if (model == "KannalaBrandt8") {
        cameraType_ = KannalaBrandt;
        camera1_ = KannalaBrandt8(readFloat("Camera1.fx"), readFloat("Camera1.fy"), readFloat("Camera1.cx"),
                                  readFloat("Camera1.cy"), readFloat("Camera1.k1"), readFloat("Camera1.k2"),
                                  readFloat("Camera1.k3"), readFloat("Camera1.k4"));
    } else {
        throw std::runtime_error("Settings: unknown Camera.type " + model);
    }
    width_ = readInt("Camera.width");
    height_ = readInt("Camera.height");
    fps_ = (float)readInt("Camera.fps");   // readParameter<int> (Settings.cc:410) into the float member
    // readORB (Settings.cc:443-451)
    nFeatures_ = readInt("ORBextractor.nFeatures");
    scaleFactor_ = readFloat("ORBextractor.scaleFactor");
    nLevels_ = readInt("ORBextractor.nLevels");
    initThFAST_ = readInt("ORBextractor.iniThFAST");
    minThFAST_ = readInt("ORBextractor.minThFAST");
}

float Settings::readFloat(const std::string& k, bool required) const {
    auto it = kv_.find(k);
    if (it == kv_.end()) {
        if (required) throw std::runtime_error("Settings: missing required parameter " + k);
        return 0.f;
    }
    errno = 0;
    char* end = nullptr;
    const double v = std::strtod(it->second.c_str(), &end);   // FileNode real (double), then (float)
    if (end == it->second.c_str() || *end != '\0' || errno)
        throw std::runtime_error("Settings: " + k + " is not a real");
    return (float)v;
}

int Settings::readInt(const std::string& k, bool required) const {
    auto it = kv_.find(k);
    if (it == kv_.end()) {
        if (required) throw std::runtime_error("Settings: missing required parameter " + k);
        return 0;
    }
    char* end = nullptr;
    const long v = std::strtol(it->second.c_str(), &end, 10);
    if (end == it->second.c_str() || *end != '\0') throw std::runtime_error("Settings: " + k + " is not an integer");
    return (int)v;
}

std::string Settings::readString(const std::string& k, bool required) const {
    auto it = kv_.find(k);
    if (it == kv_.end()) {
        if (required) throw std::runtime_error("Settings: missing required parameter " + k);
        return "";
    }
    return it->second;
}

std::unique_ptr<ORBextractor> Settings::makeORBextractor(int device) const {
    return std::unique_ptr<ORBextractor>(
        new ORBextractor(nFeatures_, scaleFactor_, nLevels_, initThFAST_, minThFAST_, device));
}

}  // namespace MAM3SLAM
