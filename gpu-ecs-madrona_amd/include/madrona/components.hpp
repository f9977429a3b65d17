// Base components (reference include/madrona/components.hpp, src/core/base.cpp).
#pragma once

#include <madrona/math.hpp>

namespace madrona {

class ECSRegistry;

namespace base {

struct Position : math::Vector3 {
    Position() = default;
    MW_INLINE Position(math::Vector3 v) : Vector3(v) {}
};

struct Rotation : math::Quat {
    Rotation() = default;
    MW_INLINE Rotation(math::Quat q) : Quat(q) {}
};

struct Scale : math::Diag3x3 {
    Scale() = default;
    MW_INLINE Scale(math::Diag3x3 d) : Diag3x3(d) {}
};

struct ObjectID {
    int32_t idx;
};

void registerTypes(ECSRegistry &registry);

}
}
