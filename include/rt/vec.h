/*
 * rt/vec.h — the reference's vector API (/root/reference/vec.h:12-40), kept name-for-name
 * so host code written against it compiles unchanged: class vec3 {double x,y,z} with
 * length / length_squared / normalize / + - * / print and the static linear_interp,
 * reflect, dot, cross; aliases point3 and RGB.
 *
 * Semantics follow vec.cpp:1-62 exactly (normalize divides by length() with no zero
 * guard; reflect normalises both arguments; linear_interp is a + t*(b-a) per component).
 * Unlike the reference the bodies are inline, so the compiler sees through them
 * (the reference's out-of-line calls cost a call per operator: SURVEY §2).
 */
#ifndef RT_VEC_H
#define RT_VEC_H

#include <cmath>
#include <iostream>

class vec3 {
public:
    double x, y, z;

    vec3() : x{0}, y{0}, z{0} {}
    vec3(double x_val, double y_val, double z_val) : x{x_val}, y{y_val}, z{z_val} {}

    double length_squared() const { return x * x + y * y + z * z; }
    double length() const { return std::sqrt(length_squared()); }
    vec3 normalize() const { return *this / length(); }

    vec3 operator+(const vec3 o) const { return vec3(x + o.x, y + o.y, z + o.z); }
    vec3 operator-() const { return vec3(-x, -y, -z); }
    vec3 operator-(const vec3 o) const { return vec3(x - o.x, y - o.y, z - o.z); }
    vec3 operator*(const vec3 o) const { return vec3(x * o.x, y * o.y, z * o.z); }
    vec3 operator*(const double s) const { return vec3(x * s, y * s, z * s); }
    vec3 operator/(const double s) const { return vec3(x / s, y / s, z / s); }
    void print() const { std::cout << x << " " << y << " " << z << " " << std::endl; }

    static double dot(const vec3 a, const vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
    static vec3 cross(const vec3& a, const vec3& b) {
        return vec3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
    }
    static vec3 linear_interp(const vec3 a, const vec3 b, double t) {
        return vec3(a.x + t * (b.x - a.x), a.y + t * (b.y - a.y), a.z + t * (b.z - a.z));
    }
    static vec3 reflect(const vec3 v, const vec3 normal) {
        const vec3 n = normal.normalize();
        const vec3 u = v.normalize();
        const double k = 2 * dot(u, n);
        return u - n * k;
    }
};

using point3 = vec3;
using RGB = vec3;

#endif
