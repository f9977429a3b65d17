"""ctypes bindings for the oracle libraries (TEST INFRASTRUCTURE ONLY).

oracle/_build/liborc.so      -- our C++ restatement of the reference path
oracle/_ref/libmadrona_ref.so -- the reference itself (built from /root/reference)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORC_PATH = os.environ.get("MADRONA_ORC_LIB") or os.path.join(ROOT, "oracle", "_build", "liborc.so")
REF_PATH = os.path.join(ROOT, "oracle", "_ref", "libmadrona_ref.so")


class PhysConfig(ctypes.Structure):
    _fields_ = [
        ("numCubes", ctypes.c_int32),
        ("numSubsteps", ctypes.c_int32),
        ("deltaT", ctypes.c_float),
        ("gravityZ", ctypes.c_float),
        ("maxContacts", ctypes.c_int32),
        ("cubeInvMass", ctypes.c_float),
        ("cubeInvInertia", ctypes.c_float),
        ("muS", ctypes.c_float),
        ("muD", ctypes.c_float),
        ("numJoints", ctypes.c_int32),
        ("numHingeJoints", ctypes.c_int32),
    ]


def default_phys_config(num_cubes=128, num_substeps=4, max_contacts=4096):
    return PhysConfig(num_cubes, num_substeps, 1.0 / 60.0, -9.8, max_contacts,
                      1.0, 1.5, 0.5, 0.5)


# Per-body record (matches RefBodyState / OrcBodyState): 38 x 4 bytes.
BODY_DTYPE = np.dtype([
    ("gen", np.uint32), ("id", np.int32),
    ("pos", np.float32, 3), ("rot", np.float32, 4), ("vel", np.float32, 6),
    ("prevPos", np.float32, 3), ("prevRot", np.float32, 4),
    ("presolvePos", np.float32, 3), ("presolveRot", np.float32, 4),
    ("presolveVel", np.float32, 6),
    ("leafID", np.int32), ("objID", np.int32), ("responseType", np.uint32),
])
assert BODY_DTYPE.itemsize == 152

CONTACT_DTYPE = np.dtype([
    ("ref", np.uint32, 2), ("alt", np.uint32, 2), ("points", np.float32, (4, 4)),
    ("numPoints", np.int32), ("normal", np.float32, 3), ("lambdaN", np.float32, 4),
])
assert CONTACT_DTYPE.itemsize == 112

BVH_NODE_DTYPE = np.dtype([
    ("minX", np.float32, 4), ("minY", np.float32, 4), ("minZ", np.float32, 4),
    ("maxX", np.float32, 4), ("maxY", np.float32, 4), ("maxZ", np.float32, 4),
    ("children", np.int32, 4), ("parentID", np.int32),
])
assert BVH_NODE_DTYPE.itemsize == 116


def _vp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def gen_collisions_inits(num_worlds, num_cubes=128, seed=0):
    lib = load_orc()
    pos = np.zeros((num_worlds, num_cubes, 3), np.float32)
    rot = np.zeros((num_worlds, num_cubes, 4), np.float32)
    lib.orc_gen_collisions_inits(num_worlds, num_cubes, ctypes.c_uint32(seed),
                                 _vp(pos), _vp(rot))
    return pos, rot


def parse_obj(path):
    """OBJ -> (positions f32[V,3], face_counts i32[F], indices u32[sum]) the way
    the reference importer hands a mesh to PhysicsLoader::loadHullFromDisk
    (src/common/importer.cpp:35-439): 'v'/'vn'/'vt' records, 'f' records of
    pos[/uv[/normal]] 1-based indices; the mesh is un-indexed and re-indexed
    by unique (position, normal, uv) bit patterns in order of first use, the
    remap meshoptimizer's generateVertexRemapMulti computes (meshoptimizer is
    an empty submodule in the reference, so this restates its published
    algorithm).  Single-mesh files only, as loadHullFromDisk asserts."""
    pos, nrm, uvs, idx, counts = [], [], [], [], []
    with open(path) as f:
        for line in f:
            t = line.split()
            if not t or t[0].startswith("#"):
                continue
            if t[0] == "v":
                pos.append(np.array(t[1:4], np.float32))
            elif t[0] == "vn":
                nrm.append(np.array(t[1:4], np.float32))
            elif t[0] == "vt":
                uvs.append(np.array(t[1:3], np.float32))
            elif t[0] == "f":
                for c in t[1:]:
                    p = (c.split("/") + ["", ""])[:3]
                    idx.append(tuple(int(x) if x else 0 for x in (p[0], p[2], p[1])))
                counts.append(len(t) - 1)
    remap, verts, out_idx = {}, [], []
    for p, n, u in idx:
        key = pos[p - 1].tobytes() + (nrm[n - 1].tobytes() if n else b"") + \
            (uvs[u - 1].tobytes() if u else b"")
        if key not in remap:
            remap[key] = len(verts)
            verts.append(pos[p - 1])
        out_idx.append(remap[key])
    return (np.array(verts, np.float32).reshape(-1, 3), np.array(counts, np.int32),
            np.array(out_idx, np.uint32))


class HullSet:
    """Packed geometry of several hulls, the argument block of
    orc_phys_create_hulls / ref_phys_create_hulls."""

    def __init__(self, meshes):
        self.meshes = list(meshes)
        self.num_verts = np.array([len(m[0]) for m in self.meshes], np.int32)
        self.num_faces = np.array([len(m[1]) for m in self.meshes], np.int32)
        self.verts = np.ascontiguousarray(np.concatenate([m[0] for m in self.meshes]), np.float32)
        self.face_counts = np.ascontiguousarray(np.concatenate([m[1] for m in self.meshes]),
                                                np.int32)
        self.indices = np.ascontiguousarray(np.concatenate([m[2] for m in self.meshes]), np.uint32)

    @classmethod
    def from_files(cls, paths):
        return cls(parse_obj(p) for p in paths)

    def args(self):
        return (len(self.meshes), _vp(self.num_verts), _vp(self.verts), _vp(self.num_faces),
                _vp(self.face_counts), _vp(self.indices))


def build_hull(mesh, lib=None):
    """HalfEdgeMesh::construct + AABB of one parsed mesh on the oracle
    (orc_build_hull) or, with lib=load_ref(), on the reference
    (ref_build_hull)."""
    lib = lib or load_orc()
    fn = lib.orc_build_hull if hasattr(lib, "orc_build_hull") else lib.ref_build_hull
    fn.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32] + [ctypes.c_void_p] * 9
    verts, counts, idx = (np.ascontiguousarray(a) for a in mesh)
    cap = 2 * int(counts.sum()) + 8
    c = np.zeros(4, np.int32)
    vo = np.zeros((len(verts), 3), np.float32)
    po = np.zeros((len(counts), 4), np.float32)
    he = np.zeros((cap, 4), np.uint32)
    polys = np.zeros(len(counts), np.uint32)
    edges = np.zeros(cap, np.uint32)
    aabb = np.zeros((2, 3), np.float32)
    fn(len(verts), _vp(verts), len(counts), _vp(counts), _vp(idx), _vp(c), _vp(vo), _vp(po),
       _vp(he), _vp(polys), _vp(edges), _vp(aabb))
    return {"vertices": vo[:c[0]], "planes": po[:c[1]], "half_edges": he[:c[3]],
            "polygons": polys[:c[1]], "edges": edges[:c[2]], "aabb": aabb}


_HULL_ARGTYPES = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_void_p]

_ORC = None
_REF = {}


def _qmul(a, b):
    w1, x1, y1, z1 = np.moveaxis(a, -1, 0)
    w2, x2, y2, z2 = np.moveaxis(b, -1, 0)
    return np.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
                     w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                     w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], axis=-1)


def _qrot(q, v):
    p = q[..., 1:]
    v = np.broadcast_to(np.asarray(v, np.float64), p.shape)
    return v + 2.0 * (np.cross(p, v) * q[..., :1] + np.cross(p, np.cross(p, v)))


def joint_inits(pos, rot, num_joints, num_hinge_joints=0):
    """Inputs for the joint workload (collisions config num_joints): cube
    2j+1 starts where joint j (cube 2j -> 2j+1) is satisfied relative to cube
    2j -- fixed: attachRot2 = 90 deg about z, r1 = (0, 1.5, 0), r2 = (0, -1.5, 0),
    separation 0.5 along the fwd axis; hinge: same rotation, 3 apart along
    local z.  Computed in float64, rounded once to float32 (an input, not a
    parity-critical computation)."""
    pos = pos.astype(np.float64).copy()
    rot = rot.astype(np.float64).copy()
    att2_inv = np.array([np.sqrt(0.5), 0.0, 0.0, -np.sqrt(0.5)])
    for j in range(num_joints):
        i1, i2 = 2 * j, 2 * j + 1
        q1, x1 = rot[:, i1], pos[:, i1]
        if j < num_joints - num_hinge_joints:
            q2 = _qmul(q1, np.broadcast_to(att2_inv, q1.shape))
            x2 = (x1 + _qrot(q1, [0, 1.5, 0]) + 0.5 * _qrot(q1, [0, 1, 0])
                  - _qrot(q2, [0, -1.5, 0]))
        else:
            q2 = q1.copy()
            x2 = x1 + _qrot(q1, [0, 0, 3.0])
        rot[:, i2] = q2
        pos[:, i2] = x2
    return pos.astype(np.float32), rot.astype(np.float32)


def load_orc():
    global _ORC
    if _ORC is None:
        lib = ctypes.CDLL(ORC_PATH)
        lib.orc_phys_create.restype = ctypes.c_void_p
        lib.orc_phys_create.argtypes = [ctypes.c_int32, ctypes.POINTER(PhysConfig),
                                        ctypes.c_void_p, ctypes.c_void_p]
        lib.orc_phys_step.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
        lib.orc_phys_read_bodies.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
        lib.orc_phys_read_bvh.argtypes = [ctypes.c_void_p, ctypes.c_int32] + [ctypes.c_void_p] * 4
        lib.orc_phys_read_candidates.argtypes = [ctypes.c_void_p, ctypes.c_int32,
                                                 ctypes.c_void_p, ctypes.c_int32]
        lib.orc_phys_read_contacts.argtypes = [ctypes.c_void_p, ctypes.c_int32,
                                               ctypes.c_void_p, ctypes.c_int32]
        lib.orc_phys_destroy.argtypes = [ctypes.c_void_p]
        lib.orc_simple_create.restype = ctypes.c_void_p
        lib.orc_simple_create.argtypes = lib.orc_phys_create.argtypes
        lib.orc_phys_create_hulls.restype = ctypes.c_void_p
        lib.orc_phys_create_hulls.argtypes = lib.orc_phys_create.argtypes + _HULL_ARGTYPES
        lib.orc_phys_ub_manifolds.restype = ctypes.c_int32
        lib.orc_phys_ub_manifolds.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        lib.orc_gen_collisions_inits.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32,
                                                 ctypes.c_void_p, ctypes.c_void_p]
        _ORC = lib
    return _ORC


def ref_available():
    return os.path.exists(REF_PATH)


def load_ref(image="main"):
    """The reference harness.  The reference's type registry is process-global
    (src/common/type_tracker.cpp:87-160: IDs in first-registration order), so
    simple_taskgraph worlds get their own image of the library
    (oracle/Makefile.ref), as each reference example is its own binary; in a
    shared image their archetype IDs would depend on which env ran first."""
    key = image
    if key not in _REF:
        path = REF_PATH if image == "main" else REF_PATH.replace(".so", f"_{image}.so")
        lib = ctypes.CDLL(path)
        lib.ref_phys_create.restype = ctypes.c_void_p
        lib.ref_phys_create.argtypes = [ctypes.c_int32, ctypes.POINTER(PhysConfig),
                                        ctypes.c_void_p, ctypes.c_void_p]
        if hasattr(lib, "ref_phys_create_hulls"):
            lib.ref_phys_create_hulls.restype = ctypes.c_void_p
            lib.ref_phys_create_hulls.argtypes = lib.ref_phys_create.argtypes + _HULL_ARGTYPES
        lib.ref_phys_step.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        lib.ref_phys_read_bodies.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
        lib.ref_phys_read_bvh.argtypes = [ctypes.c_void_p, ctypes.c_int32] + [ctypes.c_void_p] * 4
        lib.ref_phys_read_contacts.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
        if hasattr(lib, "ref_phys_read_candidates"):
            lib.ref_phys_set_candidate_log.argtypes = [ctypes.c_int32]
            lib.ref_phys_read_candidates.restype = ctypes.c_int32
            lib.ref_phys_read_candidates.argtypes = [ctypes.c_void_p, ctypes.c_int32,
                                                     ctypes.c_void_p, ctypes.c_int32]
        _REF[key] = lib
    return _REF[key]


class OraclePhys:
    """Restated CPU physics (oracle/mw_oracle.cpp)."""

    def __init__(self, cfg, pos, rot, hulls=None):
        """hulls: a HullSet -> body i uses hull i % len(hulls), the plane
        follows them (orc_phys_create_hulls); None -> the built-in cube."""
        self.lib = load_orc()
        self.cfg = cfg
        self.num_worlds = pos.shape[0]
        self.nb = cfg.numCubes + 1
        pos = np.ascontiguousarray(pos, np.float32)
        rot = np.ascontiguousarray(rot, np.float32)
        if hulls is None:
            self.h = self.lib.orc_phys_create(self.num_worlds, ctypes.byref(cfg), _vp(pos),
                                              _vp(rot))
        else:
            self.h = self.lib.orc_phys_create_hulls(self.num_worlds, ctypes.byref(cfg), _vp(pos),
                                                    _vp(rot), *hulls.args())

    def step(self, n=1, threads=1):
        self.lib.orc_phys_step(self.h, n, threads)

    def bodies(self, w):
        out = np.zeros(self.nb, BODY_DTYPE)
        self.lib.orc_phys_read_bodies(self.h, w, _vp(out))
        return out

    def bvh(self, w):
        nodes = np.zeros(4 * self.nb + 8, BVH_NODE_DTYPE)
        aabbs = np.zeros((self.nb, 6), np.float32)
        parents = np.zeros(self.nb, np.uint32)
        sorted_l = np.zeros(self.nb, np.int32)
        n = self.lib.orc_phys_read_bvh(self.h, w, _vp(nodes), _vp(aabbs), _vp(parents), _vp(sorted_l))
        return nodes[:n], aabbs, parents, sorted_l

    def candidates(self, w, cap=1 << 16):
        out = np.zeros((cap, 4), np.int32)
        n = self.lib.orc_phys_read_candidates(self.h, w, _vp(out), cap)
        return out[:n]

    def contacts(self, w):
        out = np.zeros(self.cfg.maxContacts, CONTACT_DTYPE)
        n = self.lib.orc_phys_read_contacts(self.h, w, _vp(out), self.cfg.maxContacts)
        return out[:n]

    def ub_manifolds(self, w):
        """Face manifolds so far whose reference value is undefined (an
        unwritten Manifold slot, narrowphase.cpp:828-853)."""
        return int(self.lib.orc_phys_ub_manifolds(self.h, w))

    def __del__(self):
        try:
            self.lib.orc_phys_destroy(self.h)
        except Exception:
            pass


class OracleSimple(OraclePhys):
    """simple_taskgraph worlds on the restated oracle (orc_simple_create):
    body order = Sphere rows (objects, then the test object), Agent row."""

    def __init__(self, cfg, pos, rot):
        self.lib = load_orc()
        self.lib.orc_simple_create.restype = ctypes.c_void_p
        self.cfg = cfg
        self.num_worlds = pos.shape[0]
        self.nb = cfg.numCubes + 2
        pos = np.ascontiguousarray(pos, np.float32)
        rot = np.ascontiguousarray(rot, np.float32)
        self.h = self.lib.orc_simple_create(self.num_worlds, ctypes.byref(cfg), _vp(pos), _vp(rot))


class ReferencePhys:
    """The reference itself (oracle/_ref/libmadrona_ref.so).

    log_candidates: add the harness's read-only candidate log node after the
    reference broadphase (oracle/ref_harness.cpp setupTasks) so candidates()
    returns each step's pairs; off by default (the CPU baseline)."""

    def __init__(self, cfg, pos, rot, hulls=None, log_candidates=False):
        self.lib = load_ref()
        self.lib.ref_phys_set_candidate_log(1 if log_candidates else 0)
        self.cfg = cfg
        self.num_worlds = pos.shape[0]
        self.nb = cfg.numCubes + 1
        self._pos = np.ascontiguousarray(pos, np.float32)
        self._rot = np.ascontiguousarray(rot, np.float32)
        if hulls is None:
            self.h = self.lib.ref_phys_create(self.num_worlds, ctypes.byref(cfg),
                                              _vp(self._pos), _vp(self._rot))
        else:
            self.h = self.lib.ref_phys_create_hulls(self.num_worlds, ctypes.byref(cfg),
                                                    _vp(self._pos), _vp(self._rot), *hulls.args())
        self.lib.ref_phys_set_candidate_log(0)

    def step(self, n=1):
        self.lib.ref_phys_step(self.h, n)

    def candidates(self, w, cap=1 << 16):
        """The last step's candidate pairs as (n, 4) int32 rows (Loc a, Loc b),
        the layout of OraclePhys.candidates; needs log_candidates=True."""
        out = np.zeros((cap, 4), np.int32)
        n = self.lib.ref_phys_read_candidates(self.h, w, _vp(out), cap)
        if n < 0:
            raise RuntimeError("ReferencePhys created without log_candidates")
        assert n <= cap
        return out[:n]

    def bodies(self, w):
        out = np.zeros(self.nb, BODY_DTYPE)
        self.lib.ref_phys_read_bodies(self.h, w, _vp(out))
        return out

    def bvh(self, w):
        nodes = np.zeros(4 * self.nb + 8, BVH_NODE_DTYPE)
        aabbs = np.zeros((self.nb, 6), np.float32)
        parents = np.zeros(self.nb, np.uint32)
        sorted_l = np.zeros(self.nb, np.int32)
        n = self.lib.ref_phys_read_bvh(self.h, w, _vp(nodes), _vp(aabbs), _vp(parents), _vp(sorted_l))
        return nodes[:n], aabbs, parents, sorted_l

    def contacts_raw(self, w):
        out = np.zeros(self.cfg.maxContacts, CONTACT_DTYPE)
        self.lib.ref_phys_read_contacts(self.h, w, _vp(out))
        return out

    def last_contact_count(self, w):
        """SolverData::numContacts right after the last step's last
        narrowphase node (log_candidates worlds; oracle/ref_harness.cpp
        runLogged)."""
        self.lib.ref_phys_last_contact_count.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        n = self.lib.ref_phys_last_contact_count(self.h, w)
        if n < 0:
            raise RuntimeError("no contact count (not a log_candidates world, or the node layout check failed)")
        return n


# ---------------------------------------------------------------------------
# fantasy_vs (C5): oracle/fvs_oracle.cpp and the reference ECS (oracle/ref_fvs.cpp)
# ---------------------------------------------------------------------------
FVS_ROW_DTYPE = np.dtype([("gen", np.uint32), ("id", np.int32), ("pos", np.float32, 3),
                          ("hp", np.int32), ("remaining", np.float32), ("extra", np.uint32)])


def gen_fvs_inits(num_worlds, num_dragons=50, num_knights=200, seed=0):
    lib = load_orc()
    dpos = np.zeros((num_worlds, num_dragons, 3), np.float32)
    dmana = np.zeros((num_worlds, num_dragons), np.float32)
    kpos = np.zeros((num_worlds, num_knights, 3), np.float32)
    karrows = np.zeros((num_worlds, num_knights), np.int32)
    lib.orc_gen_fvs_inits(num_worlds, num_dragons, num_knights, ctypes.c_uint32(seed),
                          _vp(dpos), _vp(dmana), _vp(kpos), _vp(karrows))
    return {"dragon_pos": dpos, "dragon_mana": dmana, "knight_pos": kpos,
            "knight_arrows": karrows}


class _FvsBase:
    prefix = None

    def __init__(self, lib, inits, first_world_index=0):
        self.lib = lib
        self.inits = {k: np.ascontiguousarray(v) for k, v in inits.items()}
        self.num_worlds, self.nd = self.inits["dragon_mana"].shape
        self.nk = self.inits["knight_arrows"].shape[1]
        create = getattr(lib, self.prefix + "_create")
        create.restype = ctypes.c_void_p
        self.h = create(self.num_worlds, self.nd, self.nk, _vp(self.inits["dragon_pos"]),
                        _vp(self.inits["dragon_mana"]), _vp(self.inits["knight_pos"]),
                        _vp(self.inits["knight_arrows"]), first_world_index)
        getattr(lib, self.prefix + "_step").argtypes = [ctypes.c_void_p, ctypes.c_int32]
        getattr(lib, self.prefix + "_read").argtypes = [ctypes.c_void_p, ctypes.c_int32,
                                                        ctypes.c_int32, ctypes.c_void_p,
                                                        ctypes.c_int32]

    def step(self, n=1):
        getattr(self.lib, self.prefix + "_step")(self.h, n)

    def table(self, w, arch):
        """Rows of Dragon (arch 0) / Knight (arch 1) in table order."""
        cap = self.nd + self.nk
        out = np.zeros(cap, FVS_ROW_DTYPE)
        n = getattr(self.lib, self.prefix + "_read")(self.h, w, arch, _vp(out), cap)
        return out[:n]


class OracleFvs(_FvsBase):
    prefix = "orc_fvs"

    def __init__(self, inits, first_world_index=0):
        super().__init__(load_orc(), inits, first_world_index)


class ReferenceFvs(_FvsBase):
    prefix = "ref_fvs"

    def __init__(self, inits, first_world_index=0):
        super().__init__(load_ref(), inits, first_world_index)


class ReferenceSimple(ReferencePhys):
    """simple_taskgraph worlds on the reference (oracle/ref_harness.cpp):
    numCubes objects + agent + test object, clamp node before physics."""

    def __init__(self, cfg, pos, rot):
        self.lib = load_ref("simple")
        self.lib.ref_simple_create.restype = ctypes.c_void_p
        self.lib.ref_simple_create.argtypes = [ctypes.c_int32, ctypes.POINTER(PhysConfig),
                                               ctypes.c_void_p, ctypes.c_void_p]
        self.cfg = cfg
        self.num_worlds = pos.shape[0]
        self.nb = cfg.numCubes + 2
        self._pos = np.ascontiguousarray(pos, np.float32)
        self._rot = np.ascontiguousarray(rot, np.float32)
        self.h = self.lib.ref_simple_create(self.num_worlds, ctypes.byref(cfg),
                                            _vp(self._pos), _vp(self._rot))


# ---------------------------------------------------------------------------
# collisions_jobs: examples/collisions' job-API toy (oracle/jobs_oracle.cpp)
# ---------------------------------------------------------------------------
JC_ROW_DTYPE = np.dtype([("gen", np.uint32), ("id", np.int32), ("pos", np.float32, 3),
                         ("rot", np.float32, 4), ("aabb", np.float32, 6)])


class OracleJobsCollisions:
    def __init__(self, pos, rot, max_candidates=1024):
        L = self.lib = load_orc()
        L.orc_jc_create.restype = ctypes.c_void_p
        L.orc_jc_create.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_void_p, ctypes.c_void_p]
        L.orc_jc_step.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.orc_jc_read.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]
        L.orc_jc_last_counts.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                         ctypes.c_void_p]
        L.orc_jc_destroy.argtypes = [ctypes.c_void_p]
        self._pos = np.ascontiguousarray(pos, np.float32)
        self._rot = np.ascontiguousarray(rot, np.float32)
        self.num_worlds, self.n = self._pos.shape[:2]
        self.h = L.orc_jc_create(self.num_worlds, self.n, max_candidates, _vp(self._pos),
                                 _vp(self._rot))

    def step(self, n=1):
        self.lib.orc_jc_step(self.h, n)

    def cubes(self, w):
        out = np.zeros(self.n, JC_ROW_DTYPE)
        k = self.lib.orc_jc_read(self.h, w, _vp(out), self.n)
        return out[:k]

    def last_counts(self, w):
        """(candidates, contacts, overflowed) of world w's last tick."""
        c = np.zeros(2, np.int32)
        flag = self.lib.orc_jc_last_counts(self.h, w, c.ctypes.data, c.ctypes.data + 4)
        return int(c[0]), int(c[1]), bool(flag)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.orc_jc_destroy(self.h)
            self.h = None
