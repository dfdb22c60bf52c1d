// Camera.h — CRT::Camera with the reference's constructor and viewport math
// (Core/Camera.cuh:13-211).  Interactive SFML input (updateCamera/updateRotation/
// updatePosition, :46-157) is out of scope; the headless equivalents are
// setYawPitch / setPosition / setSamplesPerPixel.  `toDesc()` produces the POD
// the C ABI uploads (the reference's cudaMemcpyToSymbol(d_camera), :213).
#pragma once
#include <cmath>

#include "Vec3.h"
#include "crt_hip.h"

namespace CRT {

constexpr int DEFAULT_SAMPLES_PER_PIXEL = 1;   // Camera.cuh:11

class Camera {
public:
    Camera() = default;
    // Camera.cuh:18-30 (target is accepted and ignored, like the reference)
    Camera(float aspectRatio, float fov, Vec3 position, Vec3 target, Vec3 up, float aperture, float focusDist)
        : m_AspectRatio(aspectRatio), m_VerticalFOV(fov), m_Position(position), m_Aperture(aperture),
          m_FocusDist(focusDist) {
        (void)target;
        m_WorldUp = up;
        m_SamplesPerPixel = DEFAULT_SAMPLES_PER_PIXEL;
        m_PixelSampleScale = 1.0f / m_SamplesPerPixel;
        m_Yaw = -90.0f;
        m_Pitch = 0.0f;
        updateCameraVectors();
    }

    void setSamplesPerPixel(int spp) {   // F-key high-quality mode sets 2000 (Camera.cuh:62-71)
        m_SamplesPerPixel = spp;
        m_PixelSampleScale = 1.f / m_SamplesPerPixel;
    }
    void setYawPitch(float yaw, float pitch) { m_Yaw = yaw; m_Pitch = pitch; updateCameraVectors(); }
    void setPosition(const Vec3& p) { m_Position = p; updateCameraVectors(); }
    void adjustFocusDistance(float delta) { m_FocusDist = std::fmax(0.1f, m_FocusDist + delta); updateCameraVectors(); }
    float getFocusDistance() const { return m_FocusDist; }

    void updateCameraVectors() {   // Camera.cuh:159-182
        const float PI = 3.1415926535897932385f;
        Vec3 front;
        front.e[0] = -cosf(m_Yaw * PI / 180.0f) * cosf(m_Pitch * PI / 180.0f);
        front.e[1] = -sinf(m_Pitch * PI / 180.0f);
        front.e[2] = -sinf(m_Yaw * PI / 180.0f) * cosf(m_Pitch * PI / 180.0f);
        m_Front = unitVector(front);
        m_Right = unitVector(cross(m_Front, m_WorldUp));
        m_Up = unitVector(cross(m_Right, m_Front));
        float theta = m_VerticalFOV * PI / 180.0f;
        float h = tanf(theta / 2.0f);
        float viewportHeight = 2.0f * h;
        float viewportWidth = m_AspectRatio * viewportHeight;
        m_Horizontal = m_FocusDist * viewportWidth * m_Right;
        m_Vertical = m_FocusDist * viewportHeight * m_Up;
        m_LowerLeftCorner = m_Position - m_Horizontal / 2.0f - m_Vertical / 2.0f - m_FocusDist * m_Front;
        m_LensRadius = m_Aperture / 2.0f;
    }

    crt_camera_desc toDesc() const {
        crt_camera_desc d{};
        const Vec3* src[6] = {&m_Position, &m_LowerLeftCorner, &m_Horizontal, &m_Vertical, &m_Right, &m_Up};
        float* dst[6] = {d.origin, d.lower_left, d.horizontal, d.vertical, d.right, d.up};
        for (int i = 0; i < 6; ++i)
            for (int c = 0; c < 3; ++c) dst[i][c] = src[i]->e[c];
        d.lens_radius = m_LensRadius;
        d.samples_per_pixel = m_SamplesPerPixel;
        d.pixel_sample_scale = m_PixelSampleScale;
        return d;
    }

public:
    int m_SamplesPerPixel = DEFAULT_SAMPLES_PER_PIXEL;
    float m_PixelSampleScale = 1.0f;

private:
    float m_AspectRatio = 1.f, m_VerticalFOV = 90.f;
    Vec3 m_Position;
    float m_Aperture = 0.f, m_FocusDist = 1.f;
    Vec3 m_Front, m_Up, m_Right, m_WorldUp;
    float m_Yaw = -90.f, m_Pitch = 0.f;
    Vec3 m_LowerLeftCorner, m_Horizontal, m_Vertical;
    float m_LensRadius = 0.f;
};

}  // namespace CRT
