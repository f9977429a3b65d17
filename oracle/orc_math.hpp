// ORACLE (test infrastructure only) — scalar float restatement of the
// reference math library, include/madrona/math.hpp.  Every operator keeps the
// reference's evaluation order (left-to-right sums, scalar division done as
// multiply-by-reciprocal, Quat product term order) because XPBD parity is
// decided at the ULP level.  Build with -ffp-contract=off, no -ffast-math.
#pragma once

#include <cfloat>
#include <cmath>
#include <cstdint>

namespace orc {

// glibc/x86 fminf/fmaxf for non-NaN operands: "x < y ? x : y" (ties -> y).
inline float fmin_ref(float a, float b) { return (a < b || std::isnan(b)) ? a : b; }
inline float fmax_ref(float a, float b) { return (a > b || std::isnan(b)) ? a : b; }

struct V3 {
    float x, y, z;

    float dot(const V3 &o) const { return x * o.x + y * o.y + z * o.z; }
    V3 cross(const V3 &o) const {
        return { y * o.z - z * o.y, z * o.x - x * o.z, x * o.y - y * o.x };
    }
    float length2() const { return x * x + y * y + z * z; }
    float length() const { return sqrtf(length2()); }
    float invLength() const { return 1.f / length(); }         // math.hpp:239-247
    V3 normalize() const { return *this * invLength(); }       // math.hpp:259-262
    float distance2(const V3 &o) const { return (*this - o).length2(); }

    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }

    V3 &operator+=(const V3 &o) { x += o.x; y += o.y; z += o.z; return *this; }
    V3 &operator-=(const V3 &o) { x -= o.x; y -= o.y; z -= o.z; return *this; }
    V3 &operator*=(float o) { x *= o; y *= o; z *= o; return *this; }
    V3 &operator/=(float o) { float inv = 1.f / o; return *this *= inv; }   // :342-347

    friend V3 operator-(V3 v) { return { -v.x, -v.y, -v.z }; }
    friend V3 operator+(V3 a, const V3 &b) { a += b; return a; }
    friend V3 operator-(V3 a, const V3 &b) { a -= b; return a; }
    friend V3 operator*(V3 a, float b) { a *= b; return a; }
    friend V3 operator*(float a, V3 b) { return b * a; }
    friend V3 operator/(V3 a, float b) { a /= b; return a; }

    static V3 min(V3 a, V3 b) { return { fmin_ref(a.x, b.x), fmin_ref(a.y, b.y), fmin_ref(a.z, b.z) }; }
    static V3 max(V3 a, V3 b) { return { fmax_ref(a.x, b.x), fmax_ref(a.y, b.y), fmax_ref(a.z, b.z) }; }
    static V3 zero() { return { 0, 0, 0 }; }
};

inline float dot(V3 a, V3 b) { return a.dot(b); }
inline V3 cross(V3 a, V3 b) { return a.cross(b); }

struct Q {
    float w, x, y, z;

    float length2() const { return w * w + x * x + y * y + z * z; }
    float invLength() const { return 1.f / sqrtf(length2()); }   // math.hpp:508-515
    Q normalize() const {
        float il = invLength();
        return { w * il, x * il, y * il, z * il };
    }
    Q inv() const { return { w, -x, -y, -z }; }
    V3 rotateVec(V3 v) const {                                     // math.hpp:539-548
        V3 pure { x, y, z };
        float scalar = w;
        V3 pxv = cross(pure, v);
        V3 pxpxv = cross(pure, pxv);
        return v + 2.f * ((pxv * scalar) + pxpxv);
    }
    static Q fromAngularVec(V3 v) { return { 0, v.x, v.y, v.z }; }

    Q &operator+=(Q o) { w += o.w; x += o.x; y += o.y; z += o.z; return *this; }
    Q &operator-=(Q o) { w -= o.w; x -= o.x; y -= o.y; z -= o.z; return *this; }
    friend Q operator+(Q a, Q b) { return a += b; }
    friend Q operator-(Q a, Q b) { return a -= b; }
    friend Q operator*(Q a, Q b) {                                 // math.hpp:707-715
        return {
            (a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z),
            (a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y),
            (a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x),
            (a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w),
        };
    }
};

struct Diag3 {
    float d0, d1, d2;
    Diag3 inv() const { return { 1.f / d0, 1.f / d1, 1.f / d2 }; }
    friend V3 operator*(Diag3 d, V3 v) { return { d.d0 * v.x, d.d1 * v.y, d.d2 * v.z }; }
};

struct M3 {
    V3 cols[3];

    static M3 fromQuat(Q r) {                                      // math.hpp:804-833
        float x2 = r.x * r.x, y2 = r.y * r.y, z2 = r.z * r.z;
        float xz = r.x * r.z, xy = r.x * r.y, yz = r.y * r.z;
        float wx = r.w * r.x, wy = r.w * r.y, wz = r.w * r.z;
        return {{
            { 1.f - 2.f * (y2 + z2), 2.f * (xy + wz), 2.f * (xz - wy) },
            { 2.f * (xy - wz), 1.f - 2.f * (x2 + z2), 2.f * (yz + wx) },
            { 2.f * (xz + wy), 2.f * (yz - wx), 1.f - 2.f * (x2 + y2) },
        }};
    }
    static M3 fromRS(Q r, Diag3 s) {                               // math.hpp:835-866
        float x2 = r.x * r.x, y2 = r.y * r.y, z2 = r.z * r.z;
        float xz = r.x * r.z, xy = r.x * r.y, yz = r.y * r.z;
        float wx = r.w * r.x, wy = r.w * r.y, wz = r.w * r.z;
        Diag3 ds { 2.f * s.d0, 2.f * s.d1, 2.f * s.d2 };
        return {{
            { s.d0 - ds.d0 * (y2 + z2), ds.d0 * (xy + wz), ds.d0 * (xz - wy) },
            { ds.d1 * (xy - wz), s.d1 - ds.d1 * (x2 + z2), ds.d1 * (yz + wx) },
            { ds.d2 * (xz + wy), ds.d2 * (yz - wx), s.d2 - ds.d2 * (x2 + y2) },
        }};
    }
    V3 operator*(V3 v) const { return cols[0] * v.x + cols[1] * v.y + cols[2] * v.z; }
    friend M3 operator*(const M3 &m, Diag3 d) {
        return {{ m.cols[0] * d.d0, m.cols[1] * d.d1, m.cols[2] * d.d2 }};
    }
};

struct AABB {
    V3 pMin, pMax;

    bool overlaps(const AABB &o) const {                           // math.hpp:999-1007
        return pMin.x < o.pMax.x && o.pMin.x < pMax.x &&
               pMin.y < o.pMax.y && o.pMin.y < pMax.y &&
               pMin.z < o.pMax.z && o.pMin.z < pMax.z;
    }
    AABB applyTRS(const V3 &t, const Q &r, const Diag3 &s) const { // math.hpp:1071-1103
        M3 rm = M3::fromRS(r, s);
        AABB o;
        for (int i = 0; i < 3; i++) {
            o.pMin[i] = o.pMax[i] = t[i];
            for (int j = 0; j < 3; j++) {
                float e = rm.cols[j][i] * pMin[j];
                float f = rm.cols[j][i] * pMax[j];
                if (e < f) { o.pMin[i] += e; o.pMax[i] += f; }
                else { o.pMin[i] += f; o.pMax[i] += e; }
            }
        }
        return o;
    }
    static AABB invalid() {
        return { { FLT_MAX, FLT_MAX, FLT_MAX }, { -FLT_MAX, -FLT_MAX, -FLT_MAX } };
    }
    static AABB merge(const AABB &a, const AABB &b) {
        return { V3::min(a.pMin, b.pMin), V3::max(a.pMax, b.pMax) };
    }
};

}
