// Small geometry/value types of the vacv API (reference:
// src/common/vision_structs.h).  Only VRect and VPoint are used by the pixel
// operators; the rest are kept so application code that names them compiles.
#ifndef VISION_STRUCT_H
#define VISION_STRUCT_H

namespace vision {

class VPoint {
public:
    VPoint() : x(0.0F), y(0.0F) {}
    VPoint(float px, float py) : x(px), y(py) {}
    void copy(const VPoint& o) { *this = o; }
    void clear() { x = y = 0.0F; }
    void operator+=(const VPoint& o) { x += o.x; y += o.y; }
    void operator-=(const VPoint& o) { x -= o.x; y -= o.y; }
    void operator/=(float v) { x /= v; y /= v; }
    friend VPoint operator+(VPoint a, const VPoint& b) { a += b; return a; }
    friend VPoint operator-(VPoint a, const VPoint& b) { a -= b; return a; }
    float x, y;
};

class VPoint3 {
public:
    VPoint3() : x(0.0F), y(0.0F), z(0.0F) {}
    VPoint3(float px, float py, float pz) : x(px), y(py), z(pz) {}
    void copy(const VPoint3& o) { *this = o; }
    void clear() { x = y = z = 0.0F; }
    float x, y, z;
};

class VAngle {
public:
    VAngle() : yaw(0.0F), pitch(0.0F), roll(0.0F) {}
    VAngle(float a, float b, float r) : yaw(a), pitch(b), roll(r) {}
    void copy(const VAngle& o) { *this = o; }
    void clear() { yaw = pitch = roll = 0.0F; }
    float yaw, pitch, roll;
};

class VEyeInfo {
public:
    VEyeInfo() : x(0), y(0), width(0), height(0) {}
    VEyeInfo(float px, float py, float pw, float ph) : x(px), y(py), width(pw), height(ph) {}
    void copy(const VEyeInfo& o) { x = o.x; y = o.y; width = o.width; height = o.height; }
    void clear() { x = y = width = height = 0; }
    float x, y, width, height;
    VPoint _eye_center;
    VPoint _eye_centroid;
};

class VMatrix {
public:
    VMatrix() : x(0.0F), y(0.0F), z(0.0F) {}
    VMatrix(float px, float py, float pz) : x(px), y(py), z(pz) {}
    void copy(const VMatrix& o) { *this = o; }
    void clear() { x = y = z = 0.0F; }
    float x, y, z;
};

/// ROI in pixels; crop truncates each edge to int (crop.cpp:128-131)
struct VRect {
    float left, top, right, bottom;
    VRect(float l, float t, float r, float b) : left(l), top(t), right(r), bottom(b) {}
    void set(float l, float t, float r, float b) { left = l; top = t; right = r; bottom = b; }
    float width() const { return right - left; }
    float height() const { return bottom - top; }
    bool contains(float px, float py) const {
        return left < right && top < bottom && px >= left && px < right && py >= top && py < bottom;
    }
};

struct SimpleSize { float width, height; };
struct ExtreSize { int x_min, y_min, x_max, y_max; };
struct IndexValue { int index; float value; };

enum model_class_type { param = 1, bin = 2, txt = 3 };
enum VSlidingState { NON, START, ONGOING, END };

struct VState {
    int state, continue_time, trigger_count;
    VState() { clear(); }
    void clear() { state = continue_time = trigger_count = -1; }
    void copy(const VState& o) { *this = o; }
};

struct VisGesture { int label; float confidence, x1, y1, x2, y2; };

enum NORMAL_ALG { MUL, DIV };

}  // namespace vision

#endif  // VISION_STRUCT_H
