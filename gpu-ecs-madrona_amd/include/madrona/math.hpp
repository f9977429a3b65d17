// Vector / quaternion / AABB math for the MI355X framework (host + gfx950).
//
// API and floating-point evaluation order follow the reference
// include/madrona/math.hpp (Vector3 :195-449, Quat :492-730, Diag3x3 :732-799,
// Mat3x3 :801-914, Mat3x4 :916-983, AABB :989-1128) so that the HIP kernels
// reproduce the reference CPU executor bit for bit:
//   * sums are left-to-right, scalar division is multiply-by-reciprocal,
//   * normalize() is x * (1 / sqrtf(len2)) (the reference CPU path, never rsqrt),
//   * fminf/fmaxf keep glibc's "x < y ? x : y" tie rule (ties -> second arg),
//   * everything is compiled with -ffp-contract=off (no FMA contraction) and
//     HIP's correctly rounded fp32 divide / sqrt.
#pragma once

#include <madrona/hd.hpp>

#include <cfloat>
#include <cmath>

namespace madrona {
namespace math {

constexpr inline float pi { 3.14159265358979323846264338327950288f };
constexpr inline float pi_d2 { pi / 2.f };
constexpr inline float pi_m2 { pi * 2.f };

MW_INLINE float fminRef(float a, float b) { return (a < b || b != b) ? a : b; }
MW_INLINE float fmaxRef(float a, float b) { return (a > b || b != b) ? a : b; }

struct Vector2 {
    float x;
    float y;
};

struct Vector3 {
    float x;
    float y;
    float z;

    MW_INLINE float dot(const Vector3 &o) const { return x * o.x + y * o.y + z * o.z; }
    MW_INLINE Vector3 cross(const Vector3 &o) const
    {
        return Vector3 { y * o.z - z * o.y, z * o.x - x * o.z, x * o.y - y * o.x };
    }
    MW_INLINE float length2() const { return x * x + y * y + z * z; }
    MW_INLINE float length() const { return sqrtf(length2()); }
    MW_INLINE float invLength() const { return 1.f / length(); }
    MW_INLINE float distance(const Vector3 &o) const { return (*this - o).length(); }
    MW_INLINE float distance2(const Vector3 &o) const { return (*this - o).length2(); }
    [[nodiscard]] MW_INLINE Vector3 normalize() const { return *this * invLength(); }

    MW_INLINE float &operator[](CountT i) { return i == 0 ? x : (i == 1 ? y : z); }
    MW_INLINE float operator[](CountT i) const { return i == 0 ? x : (i == 1 ? y : z); }

    MW_INLINE Vector3 &operator+=(const Vector3 &o) { x += o.x; y += o.y; z += o.z; return *this; }
    MW_INLINE Vector3 &operator-=(const Vector3 &o) { x -= o.x; y -= o.y; z -= o.z; return *this; }
    MW_INLINE Vector3 &operator+=(float o) { x += o; y += o; z += o; return *this; }
    MW_INLINE Vector3 &operator-=(float o) { x -= o; y -= o; z -= o; return *this; }
    MW_INLINE Vector3 &operator*=(float o) { x *= o; y *= o; z *= o; return *this; }
    MW_INLINE Vector3 &operator/=(float o) { float inv = 1.f / o; return *this *= inv; }

    friend MW_INLINE Vector3 operator-(Vector3 v) { return Vector3 { -v.x, -v.y, -v.z }; }
    friend MW_INLINE Vector3 operator+(Vector3 a, const Vector3 &b) { a += b; return a; }
    friend MW_INLINE Vector3 operator-(Vector3 a, const Vector3 &b) { a -= b; return a; }
    friend MW_INLINE Vector3 operator+(Vector3 a, float b) { a += b; return a; }
    friend MW_INLINE Vector3 operator-(Vector3 a, float b) { a -= b; return a; }
    friend MW_INLINE Vector3 operator*(Vector3 a, float b) { a *= b; return a; }
    friend MW_INLINE Vector3 operator/(Vector3 a, float b) { a /= b; return a; }
    friend MW_INLINE Vector3 operator+(float a, Vector3 b) { return b + a; }
    friend MW_INLINE Vector3 operator-(float a, Vector3 b) { return -b + a; }
    friend MW_INLINE Vector3 operator*(float a, Vector3 b) { return b * a; }
    friend MW_INLINE Vector3 operator/(float a, Vector3 b) { return Vector3 { a / b.x, a / b.y, a / b.z }; }

    static MW_INLINE Vector3 min(Vector3 a, Vector3 b)
    {
        return Vector3 { fminRef(a.x, b.x), fminRef(a.y, b.y), fminRef(a.z, b.z) };
    }
    static MW_INLINE Vector3 max(Vector3 a, Vector3 b)
    {
        return Vector3 { fmaxRef(a.x, b.x), fmaxRef(a.y, b.y), fmaxRef(a.z, b.z) };
    }
    static constexpr MW_INLINE Vector3 zero() { return Vector3 { 0, 0, 0 }; }
};

struct Vector4 {
    float x;
    float y;
    float z;
    float w;

    MW_INLINE Vector3 xyz() const { return Vector3 { x, y, z }; }
    static MW_INLINE Vector4 fromVector3(Vector3 v, float w) { return Vector4 { v.x, v.y, v.z, w }; }
};

MW_INLINE float dot(Vector3 a, Vector3 b) { return a.dot(b); }
MW_INLINE Vector3 cross(Vector3 a, Vector3 b) { return a.cross(b); }

struct Quat {
    float w;
    float x;
    float y;
    float z;

    MW_INLINE float length2() const { return w * w + x * x + y * y + z * z; }
    MW_INLINE float length() const { return sqrtf(length2()); }
    MW_INLINE float invLength() const { return 1.f / sqrtf(length2()); }
    [[nodiscard]] MW_INLINE Quat normalize() const
    {
        float il = invLength();
        return Quat { w * il, x * il, y * il, z * il };
    }
    [[nodiscard]] MW_INLINE Quat inv() const { return Quat { w, -x, -y, -z }; }

    MW_INLINE Vector3 rotateVec(Vector3 v) const
    {
        Vector3 pure { x, y, z };
        float scalar = w;
        Vector3 pure_x_v = cross(pure, v);
        Vector3 pure_x_pure_x_v = cross(pure, pure_x_v);
        return v + 2.f * ((pure_x_v * scalar) + pure_x_pure_x_v);
    }

    static MW_INLINE Quat angleAxis(float angle, Vector3 normal)
    {
        float coshalf = cosf(angle / 2.f);
        float sinhalf = sinf(angle / 2.f);
        return Quat { coshalf, normal.x * sinhalf, normal.y * sinhalf, normal.z * sinhalf };
    }

    static MW_INLINE Quat fromAngularVec(Vector3 v) { return Quat { 0, v.x, v.y, v.z }; }

    MW_INLINE Quat &operator+=(Quat o) { w += o.w; x += o.x; y += o.y; z += o.z; return *this; }
    MW_INLINE Quat &operator-=(Quat o) { w -= o.w; x -= o.x; y -= o.y; z -= o.z; return *this; }
    MW_INLINE Quat &operator*=(float f) { w *= f; x *= f; y *= f; z *= f; return *this; }

    friend MW_INLINE Quat operator+(Quat a, Quat b) { return a += b; }
    friend MW_INLINE Quat operator-(Quat a, Quat b) { return a -= b; }
    friend MW_INLINE Quat operator*(Quat a, Quat b)
    {
        return Quat {
            (a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z),
            (a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y),
            (a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x),
            (a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w),
        };
    }
    MW_INLINE Quat &operator*=(Quat o) { return *this = (*this * o); }
    friend MW_INLINE Quat operator*(Quat a, float b) { a *= b; return a; }
    friend MW_INLINE Quat operator*(float b, Quat a) { a *= b; return a; }
};

struct Diag3x3 {
    float d0;
    float d1;
    float d2;

    MW_INLINE Diag3x3 inv() const { return Diag3x3 { 1.f / d0, 1.f / d1, 1.f / d2 }; }
    static MW_INLINE Diag3x3 fromVec(Vector3 v) { return Diag3x3 { v.x, v.y, v.z }; }
    MW_INLINE Diag3x3 &operator*=(Diag3x3 o) { d0 *= o.d0; d1 *= o.d1; d2 *= o.d2; return *this; }
    MW_INLINE Diag3x3 &operator*=(float o) { d0 *= o; d1 *= o; d2 *= o; return *this; }
    friend MW_INLINE Diag3x3 operator*(Diag3x3 a, Diag3x3 b) { a *= b; return a; }
    friend MW_INLINE Diag3x3 operator*(Diag3x3 a, float b) { a *= b; return a; }
    friend MW_INLINE Diag3x3 operator*(float a, Diag3x3 b) { b *= a; return b; }
    friend MW_INLINE Vector3 operator*(Diag3x3 d, Vector3 v) { return Vector3 { d.d0 * v.x, d.d1 * v.y, d.d2 * v.z }; }
};

struct Mat3x3 {
    Vector3 cols[3];

    static MW_INLINE Mat3x3 fromQuat(Quat r)
    {
        float x2 = r.x * r.x, y2 = r.y * r.y, z2 = r.z * r.z;
        float xz = r.x * r.z, xy = r.x * r.y, yz = r.y * r.z;
        float wx = r.w * r.x, wy = r.w * r.y, wz = r.w * r.z;
        return {{
            { 1.f - 2.f * (y2 + z2), 2.f * (xy + wz), 2.f * (xz - wy) },
            { 2.f * (xy - wz), 1.f - 2.f * (x2 + z2), 2.f * (yz + wx) },
            { 2.f * (xz + wy), 2.f * (yz - wx), 1.f - 2.f * (x2 + y2) },
        }};
    }

    static MW_INLINE Mat3x3 fromRS(Quat r, Diag3x3 s)
    {
        float x2 = r.x * r.x, y2 = r.y * r.y, z2 = r.z * r.z;
        float xz = r.x * r.z, xy = r.x * r.y, yz = r.y * r.z;
        float wx = r.w * r.x, wy = r.w * r.y, wz = r.w * r.z;
        Diag3x3 ds = 2.f * s;
        return {{
            { s.d0 - ds.d0 * (y2 + z2), ds.d0 * (xy + wz), ds.d0 * (xz - wy) },
            { ds.d1 * (xy - wz), s.d1 - ds.d1 * (x2 + z2), ds.d1 * (yz + wx) },
            { ds.d2 * (xz + wy), ds.d2 * (yz - wx), s.d2 - ds.d2 * (x2 + y2) },
        }};
    }

    MW_INLINE Vector3 &operator[](CountT i) { return cols[i]; }
    MW_INLINE Vector3 operator[](CountT i) const { return cols[i]; }
    MW_INLINE Vector3 operator*(Vector3 v) const { return cols[0] * v.x + cols[1] * v.y + cols[2] * v.z; }
    MW_INLINE Mat3x3 operator*(const Mat3x3 &o) const
    {
        return Mat3x3 {{ *this * o.cols[0], *this * o.cols[1], *this * o.cols[2] }};
    }
    friend MW_INLINE Mat3x3 operator*(const Mat3x3 &m, Diag3x3 d)
    {
        return Mat3x3 {{ m.cols[0] * d.d0, m.cols[1] * d.d1, m.cols[2] * d.d2 }};
    }
};

struct Mat3x4 {
    Vector3 cols[4];

    static MW_INLINE Mat3x4 fromTRS(Vector3 t, Quat r, Diag3x3 s = { 1.f, 1.f, 1.f })
    {
        Mat3x3 rs = Mat3x3::fromRS(r, s);
        return Mat3x4 {{ rs.cols[0], rs.cols[1], rs.cols[2], t }};
    }
    MW_INLINE Vector3 txfmPoint(Vector3 p) const
    {
        return cols[0] * p.x + cols[1] * p.y + cols[2] * p.z + cols[3];
    }
    MW_INLINE Vector3 txfmDir(Vector3 p) const { return cols[0] * p.x + cols[1] * p.y + cols[2] * p.z; }
};

struct AABB {
    Vector3 pMin;
    Vector3 pMax;

    MW_INLINE bool overlaps(const AABB &o) const
    {
        return pMin.x < o.pMax.x && o.pMin.x < pMax.x &&
               pMin.y < o.pMax.y && o.pMin.y < pMax.y &&
               pMin.z < o.pMax.z && o.pMin.z < pMax.z;
    }
    MW_INLINE bool contains(const AABB &o) const
    {
        return pMin.x <= o.pMin.x && pMin.y <= o.pMin.y && pMin.z <= o.pMin.z &&
               pMax.x >= o.pMax.x && pMax.y >= o.pMax.y && pMax.z >= o.pMax.z;
    }
    // Reference quirk kept on purpose: "else if" means a point below pMin on an
    // axis never updates pMax on that axis (math.hpp:1022-1041).
    MW_INLINE void expand(const Vector3 &p)
    {
        if (p.x < pMin.x) { pMin.x = p.x; } else if (p.x > pMax.x) { pMax.x = p.x; }
        if (p.y < pMin.y) { pMin.y = p.y; } else if (p.y > pMax.y) { pMax.y = p.y; }
        if (p.z < pMin.z) { pMin.z = p.z; } else if (p.z > pMax.z) { pMax.z = p.z; }
    }
    [[nodiscard]] MW_INLINE AABB applyTRS(const Vector3 &translation, const Quat &rotation,
                                         const Diag3x3 &scale = { 1, 1, 1 }) const
    {
        Mat3x3 rot_mat = Mat3x3::fromRS(rotation, scale);
        AABB txfmed;
#pragma unroll
        for (CountT i = 0; i < 3; i++) {
            txfmed.pMin[i] = txfmed.pMax[i] = translation[i];
#pragma unroll
            for (CountT j = 0; j < 3; j++) {
                float e = rot_mat[j][i] * pMin[j];
                float f = rot_mat[j][i] * pMax[j];
                if (e < f) {
                    txfmed.pMin[i] += e;
                    txfmed.pMax[i] += f;
                } else {
                    txfmed.pMin[i] += f;
                    txfmed.pMax[i] += e;
                }
            }
        }
        return txfmed;
    }
    static MW_INLINE AABB invalid()
    {
        return AABB { Vector3 { FLT_MAX, FLT_MAX, FLT_MAX }, Vector3 { -FLT_MAX, -FLT_MAX, -FLT_MAX } };
    }
    static MW_INLINE AABB point(const Vector3 &p) { return AABB { p, p }; }
    static MW_INLINE AABB merge(const AABB &a, const AABB &b)
    {
        return AABB { Vector3::min(a.pMin, b.pMin), Vector3::max(a.pMax, b.pMax) };
    }
};

constexpr inline Vector3 up { 0, 0, 1 };
constexpr inline Vector3 fwd { 0, 1, 0 };
constexpr inline Vector3 right { 1, 0, 0 };

}
}
