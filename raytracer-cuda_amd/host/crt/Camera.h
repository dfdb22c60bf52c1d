// Camera.h — CRT::Camera with the reference's constructor and viewport math
// (Core/Camera.cuh:13-211) and its per-frame controller updateCamera/updateRotation/
// updatePosition (:46-157).  The reference polls SFML (sf::Keyboard::isKeyPressed,
// sf::Mouse::getPosition); here the same state arrives as an InputState, so a scripted
// input stream drives the camera exactly like a user would.  `toDesc()` produces the POD
// the C ABI uploads (the reference's cudaMemcpyToSymbol(d_camera), :213).
#pragma once
#include <cmath>

#include "Vec3.h"
#include "crt_hip.h"

namespace CRT {

constexpr int DEFAULT_SAMPLES_PER_PIXEL = 1;   // Camera.cuh:11
constexpr int HIGH_QUALITY_SAMPLES_PER_PIXEL = 2000;   // Camera.cuh:66

// What the reference polls each frame (Camera.cuh:52, :136-147; WindowManager.h:49-67).
struct InputState {
    bool keyW = false, keyA = false, keyS = false, keyD = false;   // move along -front / -right / +front / +right
    bool keySpace = false, keyLControl = false;                    // +/- world up
    bool keyF = false;                                             // held: toggles high-quality mode every frame
    bool rightMouse = false;                                       // rotation while pressed
    float mouseX = 0.f, mouseY = 0.f;                              // window coordinates
    int focusSteps = 0;                                            // PageUp (+1) / PageDown (-1) presses
};

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

    // Camera.cuh:46-72.  deltaTime in seconds.
    void updateCamera(float deltaTime, int windowWidth, int windowHeight, const InputState& in) {
        updateRotation(deltaTime, windowWidth, windowHeight, in.mouseX, in.mouseY, in.rightMouse);
        updatePosition(deltaTime, in);
        updateCameraVectors();
        if (in.keyF) m_HighQualityMode = !m_HighQualityMode;
        if (m_CameraRotates || m_CameraMoves) {
            m_SamplesPerPixel = DEFAULT_SAMPLES_PER_PIXEL;
            m_HighQualityMode = false;
        } else if (m_HighQualityMode) {
            m_SamplesPerPixel = HIGH_QUALITY_SAMPLES_PER_PIXEL;
        } else {
            m_SamplesPerPixel = DEFAULT_SAMPLES_PER_PIXEL;
        }
        m_PixelSampleScale = 1.f / m_SamplesPerPixel;
    }
    bool isCameraInMotion() const { return m_CameraRotates || m_CameraMoves; }   // :74-77
    bool isHighQuality() const { return m_HighQualityMode; }
    bool isMoving() const { return m_CameraMoves; }
    bool isRotating() const { return m_CameraRotates; }
    float yaw() const { return m_Yaw; }
    float pitch() const { return m_Pitch; }

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

    // Camera.cuh:88-130.  The reference keeps the smoothing state in function-local statics
    // (shared by every Camera of the process, initialised from the first call's window size);
    // here it is per camera, which is the same for the reference's single camera.
    void updateRotation(float deltaTime, int windowWidth, int windowHeight, float mouseX, float mouseY,
                        bool mousePressed) {
        (void)deltaTime;
        if (!m_RotInit) {
            m_LastX = windowWidth / 2.0f;
            m_LastY = windowHeight / 2.0f;
            m_SmoothX = m_LastX;
            m_SmoothY = m_LastY;
            m_RotInit = true;
        }
        const float smoothFactor = 0.5f;
        if (mousePressed) {
            if (m_FirstMouse) {
                m_LastX = mouseX;
                m_LastY = mouseY;
                m_SmoothX = mouseX;
                m_SmoothY = mouseY;
                m_FirstMouse = false;
                return;   // skip the first frame to avoid a jump
            }
            m_CameraRotates = true;
            m_SmoothX = m_SmoothX * (1 - smoothFactor) + mouseX * smoothFactor;
            m_SmoothY = m_SmoothY * (1 - smoothFactor) + mouseY * smoothFactor;
            float xoffset = m_SmoothX - m_LastX;
            float yoffset = m_SmoothY - m_LastY;
            m_LastX = m_SmoothX;
            m_LastY = m_SmoothY;
            xoffset *= -m_MouseSensitivity;
            yoffset *= -m_MouseSensitivity;
            m_Yaw += xoffset;
            m_Pitch += yoffset;
            m_Pitch = std::fmax(-89.0f, std::fmin(89.0f, m_Pitch));
        } else {
            m_FirstMouse = true;
            m_CameraRotates = false;
        }
    }
    // Camera.cuh:131-157
    void updatePosition(float deltaTime, const InputState& in) {
        const float velocity = m_MovementSpeed * deltaTime;
        const Vec3 prevPosition = m_Position;
        if (in.keyW) m_Position -= m_Front * velocity;
        if (in.keyS) m_Position += m_Front * velocity;
        if (in.keyA) m_Position -= m_Right * velocity;
        if (in.keyD) m_Position += m_Right * velocity;
        if (in.keySpace) m_Position += m_WorldUp * velocity;
        if (in.keyLControl) m_Position -= m_WorldUp * velocity;
        m_CameraMoves = m_Position != prevPosition;
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
    float m_MovementSpeed = 1.0f, m_MouseSensitivity = 0.2f;   // Camera.cuh:27-28
    bool m_CameraMoves = false, m_CameraRotates = false, m_HighQualityMode = false;
    // updateRotation's statics (Camera.cuh:90-95)
    bool m_RotInit = false, m_FirstMouse = true;
    float m_LastX = 0.f, m_LastY = 0.f, m_SmoothX = 0.f, m_SmoothY = 0.f;
};

}  // namespace CRT
