// Internal device-side data of the MI355X physics module.
//
// Per-world state that the reference keeps behind raw pointers inside the
// BVH / SolverData singletons (src/physics/broadphase.cpp:11-31,
// src/physics/physics.cpp:15-32) lives here as [world][...] slabs, so every
// kernel indexes one contiguous array for all worlds.
#pragma once

#include <madrona/physics.hpp>

namespace madrona::phys {

// 4-wide BVH node, byte-identical to broadphase::BVH::Node
// (include/madrona/physics.hpp:367-381).
struct BVHNode {
    float minX[4];
    float minY[4];
    float minZ[4];
    float maxX[4];
    float maxY[4];
    float maxZ[4];
    int32_t children[4];
    int32_t parentID;
};
static_assert(sizeof(BVHNode) == 116);

struct HullDev {
    int32_t vertOffset;
    int32_t numVerts;
    int32_t faceOffset;     // planes and polygons (one half edge per face)
    int32_t numFaces;
    int32_t hedgeOffset;
    int32_t numHedges;
    int32_t edgeOffset;
    int32_t numEdges;
};

// Per-edge topology of a hull, precomputed on the host from the half-edge
// mesh (the operands queryEdgeDirections gathers, narrowphase.cpp:474-540):
// the two faces sharing the edge and its two end vertices.
struct EdgeQuad {
    uint16_t face1, face2, v1, v2;
};

struct ObjDev {
    int32_t numObjects;
    int32_t maxVerts;
    int32_t maxFaces;
    int32_t maxEdges;
    RigidBodyMetadata *metadata;
    math::AABB *aabbs;
    uint32_t *types;              // CollisionPrimitive::Type
    HullDev *hulls;
    math::Vector3 *vertices;
    geometry::Plane *planes;
    geometry::HalfEdge *hedges;
    uint32_t *edges;              // half-edge index per edge
    uint32_t *polygons;           // half-edge index per face
    EdgeQuad *edgeQuads;          // per edge (same offsets as edges)
    // table sizes (entries), for the kernels that stage the geometry in LDS
    int32_t numVertsTotal, numPlanesTotal, numHedgesTotal, numPolygonsTotal, numEdgesTotal;
    // SAT edge query: row stride (maxFaces) of the per-pair Minkowski-test
    // tables in the group's staging area, 0 when they would not fit
    // (maxEdges x maxFaces > 128) and the test is evaluated per edge pair
    int32_t minkStride;
};

inline constexpr int32_t kMaxBodyArchetypes = 4;

struct BodyArch {
    int32_t archetype;
    int32_t capacity;
    int32_t slotBase;             // body slot of row 0 in the solver's LDS image
    int32_t *numRows;
    char *cols[13];               // Entity + Cols::Position..LeafID
};

// What the narrowphase filter needs of a body, in one 32-byte record per body
// slot: its world AABB of the substep and its object / primitive type (so a
// candidate resolves with one load per member instead of a chain through
// the ObjectID column and the object table).
struct BodyBox {
    math::AABB box;
    int32_t obj;
    uint32_t type;                // CollisionPrimitive::Type
};
static_assert(sizeof(BodyBox) == 32);

// One narrowphase pair that passed the AABB recheck, fully resolved by the
// filter kernel so the SAT kernel starts from a single load.
struct SatWork {
    int32_t world;
    int32_t slot;                 // survivor slot (== contact slot) in the world
    Loc a, b;                     // after runNarrowphase's type ordering
    int32_t aArch, bArch;         // body archetype index (PhysArgs::body)
    int32_t aObj, bObj;
    uint32_t test;                // type(a) | type(b)
    int32_t pad;
};
static_assert(sizeof(SatWork) == 48);

// A SatWork as the work lists store it: 16 B instead of 48.  The lists are
// written once by the filters and read once by the SAT / plane kernels (4.7 M
// entries per substep at the benchmark size, most of narrowphase's HBM
// traffic); a Loc's archetype is its body archetype's (body[arch].archetype).
// Rows and survivor slots fit 16 bits (<= 32767, physics_host.cpp), object
// ids 16 bits and body archetype indices 6 bits (checked at upload), the
// type test 3 bits.
struct PackedSatWork {
    int32_t world;
    uint32_t slotTest;            // slot | test << 16 | aArch << 19 | bArch << 25
    uint32_t rows;                // a.row | b.row << 16
    uint32_t objs;                // aObj | bObj << 16
};
static_assert(sizeof(PackedSatWork) == 16);
static_assert(kMaxBodyArchetypes <= 64, "6-bit body archetype indices");

// A narrowphase pair that needs a contact manifold, with the feature the SAT
// chose: hull-plane (from the filter), reference/incident face or edge pair
// (from the SAT kernel).
enum : int32_t { kJobNone = -1, kJobPlane = 0, kJobFace = 1, kJobEdge = 2 };

struct alignas(16) ContactJob {
    SatWork pair;
    int32_t kind;
    int32_t refIsA;               // face: the reference face belongs to hull a
    int32_t feature0;             // face: reference face; edge: edge of hull a
    int32_t feature1;             // face: incident face; edge: edge of hull b
    geometry::Plane plane;        // face: world reference plane; edge: {normal, separation}
};
static_assert(sizeof(ContactJob) == 80);

// Everything a physics kernel needs, passed by value (< 1 KB).
struct PhysArgs {
    int32_t numWorlds;
    int32_t numBodyArchs;
    BodyArch body[kMaxBodyArchetypes];
    int32_t maxBodiesPerWorld;    // sum of body archetype capacities

    broadphase::BVH *bvh;         // singleton column, [W]
    SolverData *solver;           // singleton column, [W]

    int32_t candArchetype;
    int32_t candCapacity;
    int32_t *numCands;            // [W]
    CandidateCollision *cands;    // [W][candCapacity]

    IDNode *idNodes;              // entity store, [W][idsPerWorld]
    int32_t idsPerWorld;
    int32_t *errorFlags;          // [W]

    int32_t maxLeaves;
    int32_t maxNodes;
    BVHNode *nodes;               // [W][maxNodes]
    Entity *leafEntities;         // [W][maxLeaves]
    math::AABB *leafAABBs;        // [W][maxLeaves]
    uint32_t *leafParents;        // [W][maxLeaves]
    int32_t *sortedLeaves;        // [W][maxLeaves]
    int32_t *leafOrder;           // [W][maxLeaves] leaves in BVH traversal (emission) order


    struct BodyBox *bodyBoxes;    // [W][maxBodiesPerWorld] per body slot, written by the
                                  // substep's integration: world AABB + object / type
    uint32_t *survInfo;           // [W][candCapacity] per survivor slot: the body slots of
                                  // its manifold's ref | alt << 16, kNoManifold without one
                                  // (the solver reads this instead of the Contact records)
    uint64_t *candSlots;          // [W][candCapacity] per candidate (findOverlaps): body slot
                                  // of a | arch index of a << 16 | bad-row flag << 24 |
                                  // body slot of b << 32 | arch index of b << 48
    int32_t *survCount;           // [W] survivors per world
    int32_t *solverOrder;         // [W] worlds by descending survivor count: the solver
                                  // grid's world order (heaviest blocks dispatched first)
    struct PackedSatWork *satWork; // [kNarrowBins][binCap] SAT / plane work lists: bin
                                  // w % kNarrowBins holds world w's hull-hull survivors
                                  // from its front and hull-plane survivors from its back
    int32_t *satWorkCount;        // [kNarrowBins][kBinStride] per-bin counters: [0] hull-hull,
                                  // [1] hull-plane entries this substep (one 64-bit
                                  // counter, reserveBin); the
                                  // filter appends, the integrate kernel / fused solver
                                  // tail resets
    int32_t binCap;               // entries per bin (worlds per bin x candCapacity)
    // Two list sets: substep s reads set s % 2 while its solver kernel's
    // tail (integrating substep s + 1) filters into set (s + 1) % 2.  The
    // node launches point satWork / satWorkCount at the set a kernel reads
    // and nextSatWork / nextSatWorkCount at the set it fills or resets.
    struct PackedSatWork *satWorkSet[2];
    int32_t *satWorkCountSet[2];
    struct PackedSatWork *nextSatWork;
    int32_t *nextSatWorkCount;
    ContactJob *hhJobs;           // [W * candCapacity] SAT verdict per satWork entry (written
                                  // only when the pair is not separated)
    int8_t *hhKinds;              // [W * candCapacity] the verdict's kind per entry: the
                                  // contact kernel scans these bytes, not 80-byte jobs
    int32_t contactGrid;          // persistent contact-kernel grid (blocks)
    int32_t planeGeoBytes;        // plane kernel's LDS copy of the hull tables (0: read
                                  // them from HBM; tables too large)
    int32_t clipCap;              // clip polygon capacity (2 x largest face)
    int32_t satGrid;              // persistent SAT grid (blocks)
    int32_t satGeoBytes;          // SAT kernel's LDS copy of the hull tables (0: read
                                  // them from HBM; tables too large)
    int32_t planeGrid;            // persistent plane-contact grid (blocks)
    Contact *candContacts;        // [W][candCapacity] manifold per survivor slot
    int32_t maxContacts;          // SolverData::maxContacts (reference assert)
    int32_t *contactOrder;        // [W][candCapacity] scratch: ordered contact list
    uint64_t *solverRecs;         // [W][candCapacity] solver contact records when K
                                  // exceeds the LDS-resident budget
    int32_t *solverPrevs;         // [W][candCapacity] predecessor pairs, same condition
    int32_t *lastNumContacts;     // [W] debug: contacts of the last substep
    int32_t recStride;            // solverRecs / solverPrevs entries per world
                                  // (candCapacity + maxJoints)

    // ConstraintData rows (JointConstraint column), solved after the
    // contacts of each substep (physics.cpp:650-671)
    int32_t jointCapacity;
    int32_t maxJoints;            // SolverData::maxJointConstraints
    int32_t *numJointRows;        // [W]
    JointConstraint *joints;      // [W][jointCapacity]
    int32_t *lastNumCands;        // [W] debug: candidates of the last step
    // Work units of the live-timed launches (bench roofline): after every
    // launch of a node being timed, unitProbeKernel adds [0] 1, [1] the
    // candidates, [2] the contact manifolds of that launch's substep, [3] 1 if
    // the launch also ran the next substep's integration + filter (solver) /
    // the first substep's filter (narrowphase), [4] the narrowphase's
    // survivor pairs.  mw_phys_take_units reads and zeroes them.
    unsigned long long *unitAccum;  // [kUnitSlots]

    // LDS images that do not fit a workgroup live in global slabs instead
    // (null: the kernel stages them in LDS); physics.hip upload() decides.
    char *overlapImage;           // [W][findOverlapsImageBytes] leaf image per world
    int32_t overlapDFSLeaves;     // findOverlaps: worlds with more leaves traverse the BVH
                                  // (stack DFS) instead of sweeping every leaf; -1: never
    // Traversal worlds' slabs (null unless some world can traverse): the
    // emission-order leaf image, per-leaf keys, and per body row its first
    // hit ranks, its count | wide flag and leaf id, per row chunk its total
    char *dfsImage;               // [W][maxLeaves] OrderedLeaf (48 B)
    int32_t *dfsKeys;             // [W][maxLeaves][2] entity id, rank << 1 | static
    uint16_t *dfsHits;            // [W][dfsRowCap][kOverlapBuf]
    int32_t *dfsRows;             // [W][dfsRowCap][2] count | kDfsWide, leaf id
    int32_t *dfsChunkTotals;      // [W][dfsChunks]
    int32_t dfsChunks;            // row chunks of kDfsBlock (0: no traversal kernels)
    int32_t dfsRowCap;            // dfsChunks * kDfsBlock
    int32_t refitLDSNodes;        // refitKernel's LDS node capacity: a world with more
                                  // used nodes walks its slab in place (same result)
    int32_t refitGlobal;          // refit walks the node slab in place
    char *satImage;               // [satImageBlocks][narrowphaseImageBytes] hull staging
    int32_t satImageBlocks;
    char *clipImage;              // [clipImageBlocks][contactImageBytes] clip polygons
    int32_t clipImageBlocks;
    char *solverImage;            // [solver blocks][solverImageBytes] body image per block
    uint32_t *solverLevelStats;   // [W] items | dependency levels << 16 of the world's last solve

    ObjDev objs;
};

inline constexpr uint32_t kNoManifold = 0xFFFF'FFFFu;
inline constexpr int32_t kUnitSlots = 5;      // PhysArgs::unitAccum

MW_INLINE int32_t numInternalNodes(int32_t num_leaves)   // broadphase.cpp:33-40
{
    int32_t a = (num_leaves - 1 + 2) / 3;
    return (a > 1 ? a : 1) + num_leaves;
}

// Narrowphase work-list bins (narrowphase.hip; world w in bin w % kNarrowBins).
constexpr int32_t kNarrowBins = 64;
constexpr int32_t kBinStride = 32;        // ints per bin (own cache lines): hull-hull at 0, hull-plane at 1 (one 64-bit counter), poison at 2

// Error flag bits (StateView::errorFlags)
inline constexpr int32_t kErrIDStoreFull = 1;
inline constexpr int32_t kErrTableFull = 2;
inline constexpr int32_t kErrCandidateOverflow = 4;
inline constexpr int32_t kErrContactOverflow = 8;
inline constexpr int32_t kErrBVHStack = 16;
inline constexpr int32_t kErrSolverBodies = 32;
// A data-derived index left its range (only reachable through corrupted
// state); bits 8..15 carry the site (physics_device.hpp guardIndex).
inline constexpr int32_t kErrIndexGuard = 64;
// More ConstraintData rows than SolverData::maxJointConstraints (the
// reference writes past its buffer, physics.cpp:34-40); the excess is dropped.
inline constexpr int32_t kErrJointOverflow = 128;
// A solve that the solver's level schedule treated as leaving an invariant
// static body untouched wrote it after all (a non-finite lambda): the
// world's contact order is no longer guaranteed to be the reference's.
inline constexpr int32_t kErrStaticSchedule = 1 << 21;

}
