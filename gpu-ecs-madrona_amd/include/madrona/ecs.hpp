// ECS identities (reference include/madrona/ecs.hpp:17-44, ecs.inl).
#pragma once

#include <madrona/hd.hpp>

namespace madrona {

struct Entity {
    uint32_t gen;
    int32_t id;

    static constexpr MW_INLINE Entity none() { return Entity { 0xFFFF'FFFFu, (int32_t)0xFFFF'FFFFu }; }
};

struct Loc {
    uint32_t archetype;
    int32_t row;

    MW_INLINE bool valid() const { return archetype != 0xFFFF'FFFFu; }
    static MW_INLINE Loc none() { return Loc { 0xFFFF'FFFFu, 0 }; }
};

struct WorldID {
    int32_t idx;
};

template <typename... ComponentTs>
struct Archetype {
    using Base = Archetype<ComponentTs...>;
};

class Context;

// Base of per-world user data.  World objects are built on the host and then
// copied into device memory once, so they must be relocatable (no owning
// host pointers used by device systems).
class WorldBase {
public:
    MW_INLINE WorldBase(Context &) {}
    WorldBase(const WorldBase &) = delete;
};

MW_INLINE bool operator==(Entity a, Entity b) { return a.gen == b.gen && a.id == b.id; }
MW_INLINE bool operator!=(Entity a, Entity b) { return !(a == b); }
MW_INLINE bool operator==(Loc a, Loc b) { return a.row == b.row && a.archetype == b.archetype; }
MW_INLINE bool operator!=(Loc a, Loc b) { return !(a == b); }

}
