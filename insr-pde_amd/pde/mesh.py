"""Mesh input for the elasticity model (cfg.use_mesh = True): the reference's
`meshio.read` + torchgp helpers (elasticity/model.py:75-93 `_init_mesh`, :198-207
`_sample_in_training`; elasticity/torchgp/{normalize, per_tet_volumes,
volume_weighted_distribution, random_tet, sample_volume, boundary_faces,
area_weighted_distribution, sample_surface}.py; elasticity/sampling.py:4-9), restated
without meshio / open3d:

  read_medit(path)         MEDIT ASCII .mesh (the format of elasticity/data/{bunny,spot}.mesh):
                           Vertices / Triangles / Tetrahedra blocks, 1-based indices and a
                           trailing reference tag per row (meshio's reader drops both)
  read_obj(path)           Wavefront .obj vertices + triangles (2-D meshes, e.g. woody.obj)
  normalize(V)             bounding-box centre to the origin, farthest vertex at radius 1
  boundary_faces(T)        faces of a tet mesh that belong to exactly one tet (gptoolbox order)
  MeshSampler              element table resident on the device; `sample(n)` draws n points
                           uniformly in the volume (tets, volume-weighted) or over the area
                           (triangles, area-weighted) -- the reference's Categorical draw +
                           Dirichlet(1,1,1,1) barycentrics (tets) / sqrt-warped barycentrics
                           (triangles), as searchsorted on a cumulative table + normalised
                           exponentials: same distributions, graph-capturable device ops.
"""
import numpy as np
import torch

# values per row of each MEDIT keyword block (element indices + reference tag)
_MEDIT_ROW = {"Edges": 3, "Triangles": 4, "Quadrilaterals": 5, "Tetrahedra": 5, "Hexahedra": 9, "Corners": 1,
              "Ridges": 1, "RequiredVertices": 1, "RequiredEdges": 1}


def read_medit(path):
    """Return (V (nv, dim) float64, blocks) with blocks[name] = 0-based int64 index arrays
    ('Triangles' (nf, 3), 'Tetrahedra' (nt, 4), ...)."""
    with open(path) as f:
        tok = f.read().split()
    i, n, dim = 0, len(tok), 3
    V, blocks = None, {}
    while i < n:
        key = tok[i]
        i += 1
        if key == "MeshVersionFormatted":
            i += 1
        elif key == "Dimension":
            dim = int(tok[i])
            i += 1
        elif key == "Vertices":
            cnt = int(tok[i])
            i += 1
            V = np.asarray(tok[i:i + cnt * (dim + 1)], dtype=np.float64).reshape(cnt, dim + 1)[:, :dim]
            i += cnt * (dim + 1)
        elif key in _MEDIT_ROW:
            cnt = int(tok[i])
            i += 1
            w = _MEDIT_ROW[key]
            rows = np.asarray(tok[i:i + cnt * w], dtype=np.int64).reshape(cnt, w)
            i += cnt * w
            if w > 1:
                blocks[key] = rows[:, :w - 1] - 1
        elif key == "End":
            break
        else:
            raise ValueError(f"{path}: unsupported MEDIT keyword {key!r}")
    if V is None:
        raise ValueError(f"{path}: no Vertices block")
    return V, blocks


def read_obj(path):
    """Vertices (nv, 3) float64 and triangles (nf, 3) int64 (0-based; polygons fanned)."""
    verts, faces = [], []
    with open(path) as f:
        for line in f:
            p = line.split()
            if not p:
                continue
            if p[0] == "v":
                verts.append([float(v) for v in p[1:4]])
            elif p[0] == "f":
                idx = [int(q.split("/")[0]) for q in p[1:]]
                idx = [k - 1 if k > 0 else len(verts) + k for k in idx]
                for a in range(1, len(idx) - 1):
                    faces.append([idx[0], idx[a], idx[a + 1]])
    return np.asarray(verts, np.float64), np.asarray(faces, np.int64).reshape(-1, 3)


def normalize(V):
    """elasticity/torchgp/normalize.py: centre of the bounding box to the origin, then scale
    so the farthest vertex is at distance 1.  V: (nv, d) tensor or array."""
    V = torch.as_tensor(V)
    vmax, vmin = V.max(dim=0).values, V.min(dim=0).values
    V = V - (vmax + vmin) / 2.0
    return V * (1.0 / torch.sqrt(torch.max(torch.sum(V ** 2, dim=-1))))


def tet_volumes(V, T):
    """|((v1 - v0) x (v2 - v0)) . (v3 - v0)| / 6 per tet (torchgp/per_tet_volumes.py)."""
    a, b, c = V[T[:, 1]] - V[T[:, 0]], V[T[:, 2]] - V[T[:, 0]], V[T[:, 3]] - V[T[:, 0]]
    return torch.abs(torch.sum(c * torch.linalg.cross(a, b), dim=-1)) / 6.0


def tri_areas(V, F):
    """|(v1 - v0) x (v2 - v0)| / 2 per triangle (torchgp/per_face_areas.py); 2-D vertices
    are lifted to z = 0."""
    if V.shape[1] == 2:
        V = torch.cat([V, torch.zeros_like(V[:, :1])], dim=1)
    return torch.linalg.norm(torch.linalg.cross(V[F[:, 1]] - V[F[:, 0]], V[F[:, 2]] - V[F[:, 0]]), dim=-1) * 0.5


def boundary_faces(T):
    """Faces occurring in exactly one tet, in the orientation of their first occurrence
    (torchgp/boundary_faces.py, after gptoolbox boundary_faces.m)."""
    T = np.asarray(T)
    allF = np.vstack((T[:, [3, 1, 2]], T[:, [2, 0, 3]], T[:, [1, 3, 0]], T[:, [0, 2, 1]]))
    _, first, counts = np.unique(np.sort(allF, axis=1), return_index=True, return_counts=True, axis=0)
    return allF[first[counts == 1]]


class MeshSampler:
    """Uniform samples in a tet mesh's volume (elements (k, 4)) or a triangle mesh's area
    (elements (k, 3)), element chosen with probability proportional to its measure."""

    def __init__(self, V, E, device="cpu"):
        self.device = torch.device(device)
        V = torch.as_tensor(V, dtype=torch.float64)
        E = torch.as_tensor(np.asarray(E), dtype=torch.int64)
        if E.dim() != 2 or E.shape[1] not in (3, 4):
            raise ValueError(f"elements must be (k, 3) triangles or (k, 4) tets, got {tuple(E.shape)}")
        w = tet_volumes(V, E) if E.shape[1] == 4 else tri_areas(V, E)
        if not bool(torch.all(w > 0)):  # the reference asserts positive volumes too
            raise ValueError("degenerate element (zero measure) in the mesh")
        cdf = torch.cumsum(w, 0)
        self.cdf = (cdf / cdf[-1]).to(self.device)  # float64 table: no bias toward late elements
        self.corners = V[E].to(self.device, torch.float32)  # (k, 3|4, dim) vertex coordinates per element
        self.k = E.shape[0]

    def uniforms_per_point(self):
        """Uniform [0, 1) draws one sample() point consumes when they are handed in (`uniforms`): two for
        the element (one float64 of 48 bits) and 4 (tet barycentrics) or 2 (triangle)."""
        return 2 + self.corners.shape[1] if self.corners.shape[1] == 4 else 4

    def sample(self, n, generator=None, uniforms=None):
        """n points; torch.rand draws from `generator` (None: torch's default), or the caller's
        (n, uniforms_per_point()) fp32 uniforms in [0, 1) with 24-bit resolution (the rank-keyed device
        Philox stream under data parallelism, which a hipGraph capture replays with fresh draws)."""
        if uniforms is not None:
            if tuple(uniforms.shape) != (n, self.uniforms_per_point()):
                raise ValueError(f"uniforms: ({n}, {self.uniforms_per_point()}) expected, got {tuple(uniforms.shape)}")
            ud = uniforms.to(torch.float64)
            u = ud[:, 0] + ud[:, 1] * 2.0 ** -24  # two 24-bit draws: one uniform of 48 bits
            rest = uniforms[:, 2:]
        else:
            u = torch.rand(n, device=self.device, dtype=torch.float64, generator=generator)
            rest = None
        idx = torch.searchsorted(self.cdf, u, right=True).clamp_(max=self.k - 1)
        cor = self.corners[idx]  # (n, 3|4, dim)
        if cor.shape[1] == 4:
            # Dirichlet(1, 1, 1, 1) barycentrics = normalised Exp(1) draws
            r4 = rest if rest is not None else torch.rand(n, 4, device=self.device, generator=generator)
            e = -torch.log(r4.clamp_min(1e-30))
            bary = e / e.sum(dim=1, keepdim=True)
        else:  # (1 - sqrt(r1), sqrt(r1)(1 - r2), sqrt(r1) r2)  (torchgp/sample_surface.py)
            r = rest if rest is not None else torch.rand(n, 2, device=self.device, generator=generator)
            su = torch.sqrt(r[:, :1])
            bary = torch.cat([1 - su, su * (1 - r[:, 1:]), su * r[:, 1:]], dim=1)
        return torch.sum(bary.unsqueeze(-1) * cor, dim=1)


def load_mesh(path, dim, device="cpu"):
    """elasticity/model.py:75-93: vertices (normalised, x2), volume elements (tets in 3-D,
    triangles in 2-D) and surface faces; returns (V (nv, dim) float32 on device, E, SF)."""
    if path.endswith(".mesh"):
        V, blocks = read_medit(path)
        if dim == 3:
            if "Tetrahedra" not in blocks:
                raise ValueError(f"{path}: a 3-D elasticity mesh needs a Tetrahedra block")
            E = blocks["Tetrahedra"]
            SF = boundary_faces(E)
        else:
            E = blocks["Triangles"]
            SF = E
    elif path.endswith(".obj"):
        V, E = read_obj(path)
        SF = E
    elif path.endswith(".npz"):  # a fixture derived from a .mesh (tests/golden/make_bunny_fixture.py)
        with np.load(path) as z:  # arrays only (allow_pickle stays False)
            V, E = z["V"].astype(np.float64), z["T"].astype(np.int64)
        if dim != 3 or E.shape[1] != 4:
            raise ValueError(f"{path}: a tetrahedral (3-D) mesh fixture is expected")
        SF = boundary_faces(E)
    else:
        raise ValueError(f"unsupported mesh file {path!r} (.mesh, .obj or a .npz fixture)")
    V = normalize(torch.as_tensor(V, dtype=torch.float64)) * 2.0
    return V.to(device, torch.float32), E, SF
