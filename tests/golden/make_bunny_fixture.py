"""Derive the elasticity3Dbunny mesh fixture from the reference's own data file.

    python tests/golden/make_bunny_fixture.py   # in this container (reads /root/reference)

/root/reference/elasticity/data/bunny.mesh (MEDIT ASCII, the mesh scripts/elasticity3Dbunny.sh
trains on) does not travel to the GPU box; its vertices and tetrahedra do, as data:
tests/golden/bunny_mesh.npz = {V: (nv, 3) float64 as read, T: (nt, 4) int32 0-based}.
pde/mesh.py load_mesh() reads either file the same way (normalise x2, boundary faces).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "..", "insr-pde_amd")]
from pde.mesh import read_medit  # noqa: E402

SRC = "/root/reference/elasticity/data/bunny.mesh"


def main():
    V, blocks = read_medit(SRC)
    T = blocks["Tetrahedra"].astype(np.int32)
    out = os.path.join(HERE, "bunny_mesh.npz")
    np.savez_compressed(out, V=V, T=T)
    print(out, V.shape, T.shape, os.path.getsize(out))


if __name__ == "__main__":
    main()
