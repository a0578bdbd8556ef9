/*
 * host/scene.cpp — host side of the scene API (include/rt/scene.h).
 *
 * SceneGeometry::intersect keeps the reference's semantics on the CPU (the plugin
 * interface stays usable by host code, e.g. for picking), pack() flattens objects for
 * the GPU path, and Camera keeps init() (scene.cpp:80-106, via the C-ABI restatement
 * rt_camera_init so host and GPU agree bit for bit) and the movement controls
 * (scene.cpp:108-165) that only change the camera's position/direction inputs.
 */
#include <cfloat>
#include <cmath>
#include <stdexcept>

#include "../../include/rt/scene.h"

/* A primitive type the kernels do not implement (a SceneGeometry subclass written against
 * the reference's scene.h:51-60, which has intersect() only): rt_scene reports it instead
 * of rendering something else. */
void SceneGeometry::pack(rt_prim*) const {
    throw std::invalid_argument(
        "rt_scene: unsupported primitive: this SceneGeometry subclass has no GPU record "
        "(the kernels implement Sphere and Wall; override pack())");
}

void SceneGeometry::pack_material(rt_prim* out) const {
    out->mat.color[0] = mat.color.x;
    out->mat.color[1] = mat.color.y;
    out->mat.color[2] = mat.color.z;
    out->mat.ambient = mat.ambient;
    out->mat.metallic = mat.metallic;
    out->mat.diffuse = mat.diffuse;
    out->mat.specular = mat.specular;
    out->mat.specular_exponent = mat.specular_exponent;
}

/* Wall: finite two-sided rectangle with its corner at `position`; reports the
 * PARAMETRIC ray distance t and the stored normal (scene.cpp:4-35 semantics). */
Collision Wall::intersect(ray r) const {
    const vec3 o = r.get_origin(), d = r.get_direction();
    const double t = vec3::dot(position - o, normal) / vec3::dot(normal, d);
    if (t > 0) {
        const vec3 x_axis = vec3::cross(normal, vec3(0, 0, 1)).normalize();
        const vec3 y_axis = vec3::cross(x_axis, normal).normalize();
        const vec3 rel = r.at(t) - position;
        const double u = vec3::dot(rel, x_axis), v = vec3::dot(rel, y_axis);
        if (u >= 0 && u <= length && v >= 0 && v <= width) return Collision(t, normal, true, -1);
    }
    return Collision(-1, vec3(0, 0, 0), false, -1);
}

void Wall::pack(rt_prim* out) const {
    *out = rt_prim{};
    out->kind = RT_PRIM_WALL;
    pack_material(out);
    out->position[0] = position.x;
    out->position[1] = position.y;
    out->position[2] = position.z;
    out->normal[0] = normal.x;
    out->normal[1] = normal.y;
    out->normal[2] = normal.z;
    out->length = length;
    out->width = width;
}

/* Sphere: reports the WORLD distance proj*|d| and the un-normalised normal P - C;
 * a tangent ray (det == 0) uses -b/a for the distance (scene.cpp:40-78 semantics). */
Collision Sphere::intersect(ray r) const {
    const vec3 o = r.get_origin(), d = r.get_direction();
    const vec3 oc = o - center;
    const double a = d.length_squared();
    const double b = 2 * vec3::dot(d, oc);
    const double c = oc.length_squared() - radius * radius;
    const double det = b * b - 4 * a * c;
    if (det < 0) return Collision(-1, vec3(0, 0, 0), false, -1);
    double proj;
    vec3 point;
    if (det == 0) {
        point = o + d * (-b / (2 * a));
        proj = (-b - std::sqrt(det)) / a;
    } else {
        const double root = std::sqrt(det);
        const double near_t = (-b - root) / (2 * a), far_t = (-b + root) / (2 * a);
        proj = far_t < near_t ? far_t : near_t;
        point = o + d * proj;
    }
    return Collision(proj * d.length(), point - center, true, -1);
}

void Sphere::pack(rt_prim* out) const {
    *out = rt_prim{};
    out->kind = RT_PRIM_SPHERE;
    pack_material(out);
    out->position[0] = center.x;
    out->position[1] = center.y;
    out->position[2] = center.z;
    out->radius = radius;
}

std::vector<vec3> Camera::init() {
    const double p[3] = {position.x, position.y, position.z};
    const double l[3] = {lookat.x, lookat.y, lookat.z};
    const double u[3] = {vup.x, vup.y, vup.z};
    rt_camera c;
    rt_camera_init(p, l, u, vfov, aspect_ratio, image_width, &c);
    image_height = c.height;
    focal_length = (position - lookat).length();
    const vec3 w = (position - lookat).normalize();
    direction = w;
    image_top_left = vec3(c.image_top_left[0], c.image_top_left[1], c.image_top_left[2]);
    const vec3 dx(c.pixel_delta_x[0], c.pixel_delta_x[1], c.pixel_delta_x[2]);
    const vec3 dy(c.pixel_delta_y[0], c.pixel_delta_y[1], c.pixel_delta_y[2]);
    // fov_top_left as scene.cpp:102 forms it (members only; not used by rendering)
    const double fov_h = 2 * std::tan(vfov * 3.14 / 180.0 / 2) * focal_length;
    const double fov_w = fov_h * (image_width / image_height);
    const vec3 fx = vec3::cross(vup, w).normalize() * fov_w;
    const vec3 fy = vec3::cross(w, vec3::cross(vup, w).normalize()) * (-fov_h);
    fov_top_left = position - (w * focal_length) - fx / 2 - fy / 2;
    // like the reference, the deltas are returned, the members stay as they were
    return {dx, dy};
}

vec3 Camera::forward_vec() { return direction.normalize(); }
vec3 Camera::right_vec() { return vec3::cross(direction, vup).normalize(); }
vec3 Camera::up_vec() { return vec3::cross(right_vec(), direction).normalize(); }
void Camera::forward() { position = position + forward_vec() * movement_speed; }
void Camera::backward() { position = position - forward_vec() * movement_speed; }
void Camera::right() { position = position + right_vec() * movement_speed; }
void Camera::left() { position = position - right_vec() * movement_speed; }

void Camera::rotate_left_right(double angle) {
    const double heading = std::atan2(direction.y, direction.x) + angle;
    const double planar = vec3(direction.x, direction.y, 0).length();
    direction = vec3(std::cos(heading) * planar, std::sin(heading) * planar, direction.z);
    vup = up_vec();
}

void Camera::rotate_up_down(double angle) {
    const double planar = vec3(direction.x, direction.y, 0).length();
    const double pitch = std::atan2(direction.z, planar);
    double next = pitch + angle;
    if (next > M_PI / 2) next = pitch;
    if (next < -M_PI / 2) next = -pitch;
    const vec3 flat = vec3(direction.x, direction.y, 0).normalize() * std::cos(next);
    direction = vec3(flat.x, flat.y, std::sin(next));
    vup = up_vec();
}
