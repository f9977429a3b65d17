// Rigid-body physics public API for the MI355X framework.
//
// Reference interface: include/madrona/physics.hpp:1-468 (components, Contact,
// ObjectManager, BVH, solver state, RigidBodyPhysicsSystem, Cols).  Types that
// live in ECS columns keep the reference's byte layout (Contact 112 B, BVH node
// 116 B, ...), so Locs, contacts and exported columns compare bit for bit with
// the reference CPU executor.  The step itself runs as HIP kernels over all
// worlds (csrc/physics/physics.hip); DESIGN.md §3 maps each kernel to the
// reference functions it replaces.
#pragma once

#include <madrona/components.hpp>
#include <madrona/taskgraph.hpp>

#include <utility>

namespace madrona::phys {

namespace geometry {

// Host-side polygon soup used to build hulls (geometry.cpp:14-48).
struct FastPolygonList {
    uint32_t maxIndices;
    uint32_t *buffer;
    uint32_t size;
    uint32_t edgeCount;
    uint32_t polygonCount;

    void allocate(uint32_t maxIdx);
    void free();
    void addPolygon(Span<const uint32_t> vertex_indices);

    inline uint32_t *begin() { return &buffer[1]; }
    inline uint32_t *next(uint32_t *it) { return it + it[-1] + 1; }
    inline uint32_t *end() { return buffer + size + 1; }
    inline uint32_t getPolygonVertexCount(uint32_t *it) { return it[-1]; }
};

using PolygonData = uint32_t;
using PolygonID = uint32_t;
using EdgeData = uint32_t;
using HalfEdgeID = uint32_t;
using VertexID = uint32_t;

struct HalfEdge {
    HalfEdgeID next;
    HalfEdgeID twin;
    VertexID rootVertex;
    PolygonID polygon;
};

struct Plane {
    math::Vector3 normal;
    float d;
};

struct Segment {
    math::Vector3 p1;
    math::Vector3 p2;
};

// Host-built half-edge mesh (geometry.cpp:52-194).  Pointers are host
// pointers; RigidBodyPhysicsSystem::init flattens them into the device object
// table.
class HalfEdgeMesh {
public:
    void construct(FastPolygonList &polygons, uint32_t vertexCount,
                   const math::Vector3 *vertices);

    PolygonData *mPolygons;
    Plane *mFacePlanes;
    EdgeData *mEdges;
    HalfEdge *mHalfEdges;
    math::Vector3 *mVertices;

    uint32_t mHalfEdgeCount;
    uint32_t mPolygonCount;
    uint32_t mEdgeCount;
    uint32_t mVertexCount;
};

}

struct ExternalForce : math::Vector3 {
    ExternalForce() = default;
    MW_INLINE ExternalForce(math::Vector3 v) : Vector3(v) {}
};

struct ExternalTorque : math::Vector3 {
    ExternalTorque() = default;
    MW_INLINE ExternalTorque(math::Vector3 v) : Vector3(v) {}
};

enum class ResponseType : uint32_t {
    Dynamic,
    Kinematic,
    Static,
};

struct Velocity {
    math::Vector3 linear;
    math::Vector3 angular;
};

struct CollisionEvent {
    Entity a;
    Entity b;
};

struct CandidateCollision {
    Loc a;
    Loc b;
};

struct CandidateTemporary : Archetype<CandidateCollision> {};

struct Contact {
    Loc ref;
    Loc alt;
    math::Vector4 points[4];
    int32_t numPoints;
    math::Vector3 normal;
    float lambdaN[4];
};
static_assert(sizeof(Contact) == 112);

struct CollisionEventTemporary : Archetype<CollisionEvent> {};

struct JointConstraint {
    enum class Type { Fixed, Hinge };

    struct Fixed {
        math::Quat attachRot1;
        math::Quat attachRot2;
        float separation;
    };

    struct Hinge {
        math::Vector3 a1Local;
        math::Vector3 a2Local;
        math::Vector3 b1Local;
        math::Vector3 b2Local;
    };

    Entity e1;
    Entity e2;
    Type type;
    union {
        Fixed fixed;
        Hinge hinge;
    };
    math::Vector3 r1;
    math::Vector3 r2;

    // reference include/madrona/physics.inl:151-190
    static MW_HD inline JointConstraint setupFixed(Entity e1, Entity e2,
                                                   math::Quat attach_rot1,
                                                   math::Quat attach_rot2,
                                                   math::Vector3 r1, math::Vector3 r2,
                                                   float separation)
    {
        JointConstraint j {};
        j.e1 = e1;
        j.e2 = e2;
        j.type = Type::Fixed;
        j.fixed = Fixed { attach_rot1, attach_rot2, separation };
        j.r1 = r1;
        j.r2 = r2;
        return j;
    }

    static MW_HD inline JointConstraint setupHinge(Entity e1, Entity e2,
                                                   math::Vector3 a1_local,
                                                   math::Vector3 a2_local,
                                                   math::Vector3 b1_local,
                                                   math::Vector3 b2_local,
                                                   math::Vector3 r1, math::Vector3 r2)
    {
        JointConstraint j {};
        j.e1 = e1;
        j.e2 = e2;
        j.type = Type::Hinge;
        j.hinge = Hinge { a1_local, a2_local, b1_local, b2_local };
        j.r1 = r1;
        j.r2 = r2;
        return j;
    }
};
static_assert(sizeof(JointConstraint) == 92);

struct ConstraintData : Archetype<JointConstraint> {};

struct RigidBodyMetadata {
    math::Vector3 invInertiaTensor;
    float invMass;
    float muS;
    float muD;
};

struct CollisionPrimitive {
    enum class Type : uint32_t {
        Sphere = 1 << 0,
        Hull = 1 << 1,
        Plane = 1 << 2,
    };

    struct Sphere { float radius; };
    struct Hull { geometry::HalfEdgeMesh halfEdgeMesh; };
    struct Plane {};

    Type type;
    union {
        Sphere sphere;
        Plane plane;
        Hull hull;
    };
};

// Host object table handed to RigidBodyPhysicsSystem::init (physics.hpp:275-294).
struct ObjectManager {
    RigidBodyMetadata *metadata;
    math::AABB *aabbs;
    CollisionPrimitive *primitives;
    int32_t numObjects;          // MI355X addition: table length for the upload
};

struct ObjectData {
    void *mgr;                   // device object table (opaque to user code)
};

namespace broadphase {

struct LeafID {
    int32_t id;
};

// Per-world BVH scalars (the node / leaf arrays are [world][...] slabs owned
// by the physics module, see csrc/physics/physics_impl.hpp).
struct BVH {
    int32_t numLeaves;
    int32_t maxLeaves;
    int32_t numNodes;
    int32_t usedNodes;
    int32_t forceRebuild;
    float leafVelocityExpansion;
    float leafAccelExpansion;
    int32_t worldIdx;

    MW_INLINE void rebuildOnUpdate() { forceRebuild = 1; }
    MW_INLINE void clearLeaves() { numLeaves = 0; }
};

}

namespace solver {

struct SubstepPrevState {
    math::Vector3 prevPosition;
    math::Quat prevRotation;
};

struct PreSolvePositional {
    math::Vector3 x;
    math::Quat q;
};

struct PreSolveVelocity {
    math::Vector3 v;
    math::Vector3 omega;
};

}

// Per-world solver scalars (reference SolverData, src/physics/physics_impl.hpp:7-26).
struct SolverData {
    int32_t numContacts;
    int32_t maxContacts;
    int32_t numJointConstraints;
    int32_t maxJointConstraints;
    float deltaT;
    float h;
    math::Vector3 g;
    float gMagnitude;
    float restitutionThreshold;
};

struct RigidBodyPhysicsSystem {
    static void init(Context &ctx,
                     ObjectManager *obj_mgr,
                     float delta_t,
                     CountT num_substeps,
                     math::Vector3 gravity,
                     CountT max_dynamic_objects,
                     CountT max_contacts_per_world,
                     CountT max_joint_constraints_per_world);

    static void reset(Context &ctx);
    static broadphase::LeafID registerEntity(Context &ctx, Entity e, base::ObjectID obj_id);

    static void registerTypes(ECSRegistry &registry);

    static TaskGraph::NodeID setupBroadphaseTasks(TaskGraph::Builder &builder,
                                                  Span<const TaskGraph::NodeID> deps);
    static TaskGraph::NodeID setupSubstepTasks(TaskGraph::Builder &builder,
                                               Span<const TaskGraph::NodeID> deps,
                                               CountT num_substeps);
    static TaskGraph::NodeID setupCleanupTasks(TaskGraph::Builder &builder,
                                               Span<const TaskGraph::NodeID> deps);

    // MI355X addition: upper bound on candidate pairs per world (the
    // reference's CPU table grows without bound; the device table is fixed).
    static void setMaxCandidatesPerWorld(ECSRegistry &registry, int32_t max_candidates);
};

struct Cols {
    static constexpr inline CountT Position = 1;
    static constexpr inline CountT Rotation = 2;
    static constexpr inline CountT Scale = 3;
    static constexpr inline CountT Velocity = 4;
    static constexpr inline CountT ObjectID = 5;
    static constexpr inline CountT ResponseType = 6;
    static constexpr inline CountT SubstepPrevState = 7;
    static constexpr inline CountT PreSolvePositional = 8;
    static constexpr inline CountT PreSolveVelocity = 9;
    static constexpr inline CountT ExternalForce = 10;
    static constexpr inline CountT ExternalTorque = 11;
    static constexpr inline CountT LeafID = 12;

    static constexpr inline CountT CandidateCollision = 1;
};

}
