// Vec3.h — host value types with the reference's API and arithmetic
// (Core/Vec3.cuh:8-234, Core/Interval.cuh:6-49, Core/AABB.cuh:9-189).
// Host code is compiled with -ffp-contract=off so every operation rounds
// exactly like the reference's single-precision code.
#pragma once
#include <cmath>
#include <limits>

namespace CRT {

class Vec3 {
public:
    float e[3];
    Vec3() : e{0.f, 0.f, 0.f} {}
    Vec3(float e0, float e1, float e2) : e{e0, e1, e2} {}
    explicit Vec3(float v) : e{v, v, v} {}
    float x() const { return e[0]; }
    float y() const { return e[1]; }
    float z() const { return e[2]; }
    Vec3 operator-() const { return Vec3(-e[0], -e[1], -e[2]); }
    float operator[](int i) const { return e[i]; }
    float& operator[](int i) { return e[i]; }
    bool operator==(const Vec3& v) const { return e[0] == v.e[0] && e[1] == v.e[1] && e[2] == v.e[2]; }
    bool operator!=(const Vec3& v) const { return !(*this == v); }
    Vec3& operator+=(const Vec3& v) { e[0] += v.e[0]; e[1] += v.e[1]; e[2] += v.e[2]; return *this; }
    Vec3& operator-=(const Vec3& v) { e[0] -= v.e[0]; e[1] -= v.e[1]; e[2] -= v.e[2]; return *this; }
    Vec3& operator*=(const Vec3& v) { e[0] *= v.e[0]; e[1] *= v.e[1]; e[2] *= v.e[2]; return *this; }
    Vec3& operator*=(float t) { e[0] *= t; e[1] *= t; e[2] *= t; return *this; }
    Vec3& operator/=(float t) { return *this *= 1 / t; }
    float maxComponent() const { return std::fmax(e[0], std::fmax(e[1], e[2])); }
    static Vec3 min(const Vec3& a, const Vec3& b) {
        return Vec3(std::fmin(a.e[0], b.e[0]), std::fmin(a.e[1], b.e[1]), std::fmin(a.e[2], b.e[2]));
    }
    static Vec3 max(const Vec3& a, const Vec3& b) {
        return Vec3(std::fmax(a.e[0], b.e[0]), std::fmax(a.e[1], b.e[1]), std::fmax(a.e[2], b.e[2]));
    }
    float lengthSquared() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }
    float length() const { return std::sqrt(lengthSquared()); }
};
using Point3 = Vec3;
using Color = Vec3;

inline Vec3 operator+(const Vec3& u, const Vec3& v) { return Vec3(u.e[0] + v.e[0], u.e[1] + v.e[1], u.e[2] + v.e[2]); }
inline Vec3 operator-(const Vec3& u, const Vec3& v) { return Vec3(u.e[0] - v.e[0], u.e[1] - v.e[1], u.e[2] - v.e[2]); }
inline Vec3 operator*(const Vec3& u, const Vec3& v) { return Vec3(u.e[0] * v.e[0], u.e[1] * v.e[1], u.e[2] * v.e[2]); }
inline Vec3 operator*(float t, const Vec3& v) { return Vec3(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline Vec3 operator*(const Vec3& v, float t) { return Vec3(v.e[0] * t, v.e[1] * t, v.e[2] * t); }
inline Vec3 operator/(const Vec3& v, float t) { return (1 / t) * v; }
inline float dot(const Vec3& u, const Vec3& v) { return u.e[0] * v.e[0] + u.e[1] * v.e[1] + u.e[2] * v.e[2]; }
inline Vec3 cross(const Vec3& u, const Vec3& v) {
    return Vec3(u.e[1] * v.e[2] - u.e[2] * v.e[1], u.e[2] * v.e[0] - u.e[0] * v.e[2], u.e[0] * v.e[1] - u.e[1] * v.e[0]);
}
inline Vec3 unitVector(const Vec3& v) { return v / v.length(); }

constexpr float INFINITY_CRT = std::numeric_limits<float>::infinity();

struct Interval {
    float min = INFINITY_CRT, max = -INFINITY_CRT;
    Interval() = default;
    Interval(float a, float b) : min(a), max(b) {}
    float size() const { return max - min; }
    Interval expand(float delta) const { float p = delta / 2.f; return Interval(min - p, max + p); }
};

// AABB.cuh semantics: the Interval/combine/expand(AABB) constructors pad axes
// thinner than 1e-6 by +-5e-7 (padToMinimums, :181-186); expand(Point) does not.
struct AABB {
    Interval x, y, z;
    AABB() = default;                                   // :13 — no padding
    AABB(const Interval& ix, const Interval& iy, const Interval& iz) : x(ix), y(iy), z(iz) { padToMinimums(); }
    AABB(const Point3& a, const Point3& b) {            // :28-35
        x = Interval(std::fmin(a[0], b[0]), std::fmax(a[0], b[0]));
        y = Interval(std::fmin(a[1], b[1]), std::fmax(a[1], b[1]));
        z = Interval(std::fmin(a[2], b[2]), std::fmax(a[2], b[2]));
        padToMinimums();
    }
    static AABB empty() { return AABB(Interval(), Interval(), Interval()); }   // AABB_EMPTY, :188
    void expand(const Point3& p) {                      // :51-59
        x.min = std::fmin(x.min, p.x()); x.max = std::fmax(x.max, p.x());
        y.min = std::fmin(y.min, p.y()); y.max = std::fmax(y.max, p.y());
        z.min = std::fmin(z.min, p.z()); z.max = std::fmax(z.max, p.z());
    }
    void expand(const AABB& o) {                        // :83-89
        x = Interval(std::fmin(x.min, o.x.min), std::fmax(x.max, o.x.max));
        y = Interval(std::fmin(y.min, o.y.min), std::fmax(y.max, o.y.max));
        z = Interval(std::fmin(z.min, o.z.min), std::fmax(z.max, o.z.max));
        padToMinimums();
    }
    static AABB combine(const AABB& a, const AABB& b) { // :91-98
        return AABB(Interval(std::fmin(a.x.min, b.x.min), std::fmax(a.x.max, b.x.max)),
                    Interval(std::fmin(a.y.min, b.y.min), std::fmax(a.y.max, b.y.max)),
                    Interval(std::fmin(a.z.min, b.z.min), std::fmax(a.z.max, b.z.max)));
    }
    float area() const {                                // :74-81
        float ex = x.size(), ey = y.size(), ez = z.size();
        return 2.0f * (ex * ey + ey * ez + ez * ex);
    }
    void padToMinimums() {
        const float delta = 0.000001f;
        if (x.size() < delta) x = x.expand(delta);
        if (y.size() < delta) y = y.expand(delta);
        if (z.size() < delta) z = z.expand(delta);
    }
};

}  // namespace CRT
