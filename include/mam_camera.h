/*
 * mam_camera.h — the GeometricCamera a search / solve projects with (gfx950 / MI355X C-ABI).
 *
 * Replaces the camera object the reference hands around by pointer (Frame::mpCamera, KeyFrame::mpCamera,
 * EdgeSE3ProjectXYZ::pCamera): GeometricCamera (include/CameraModels/GeometricCamera.h:95-101) with its two models
 *   Pinhole         mvParameters = {fx, fy, cx, cy}            src/CameraModels/Pinhole.cpp:35-81, 107-129
 *   KannalaBrandt8  mvParameters = {fx, fy, cx, cy, k0..k3}    src/CameraModels/KannalaBrandt8.cpp:46-175, 216-406
 * as one plain value. `model` is GeometricCamera::mnType (CAM_PINHOLE = 0, CAM_FISHEYE = 1).
 */
#ifndef MAM_CAMERA_H
#define MAM_CAMERA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MAM_CAM_PINHOLE 0          /* GeometricCamera::CAM_PINHOLE */
#define MAM_CAM_KANNALA_BRANDT8 1  /* GeometricCamera::CAM_FISHEYE */

typedef struct mam_camera {
    float fx, fy, cx, cy;   /* mvParameters[0..3] (float, as the reference stores them) */
    float k[4];             /* KannalaBrandt8 k0..k3 = mvParameters[4..7]; not read for a Pinhole */
    int32_t model;          /* MAM_CAM_* */
    float precision;        /* KannalaBrandt8::precision, unproject's Newton tolerance (1e-6 default,
                               KannalaBrandt8.h:42-47); not read for a Pinhole */
} mam_camera;

/* Round-1 name: a Pinhole is a mam_camera with model 0 (zero-initialised k / precision). */
typedef mam_camera mam_pinhole;

#ifdef __cplusplus
}
#endif
#endif /* MAM_CAMERA_H */
