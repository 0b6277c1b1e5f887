"""Copies the reference's own JCAMP-DX test files into tests/golden/jcampdx/.

Run in the build container (needs /root/reference; the GPU box does not):

    python tests/golden/make_jcampdx_fixtures.py

The files are data the reference's tests read (jcampdx.rs:1101-1224 reads
data/jcamp-dx/test/v{5,6}/*.dx; docs read data/jcamp-dx/blood/blood_01.dx),
stored gzip-compressed. ``blood_01_affn.npz`` holds the AFFN intensities of
test/v6/xydata_affn.dx, parsed here with plain ``str.split`` (independent of the
package's decoder), as the expected values for every compressed encoding.
"""
import gzip
import os
import shutil

import numpy as np

REF = "/root/reference/data/jcamp-dx"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "jcampdx")
FILES = {
    "v5_xydata_difdup.dx": "test/v5/xydata_difdup.dx",
    "v6_xydata_difdup.dx": "test/v6/xydata_difdup.dx",
    "v6_ntuples_difdup.dx": "test/v6/ntuples_difdup.dx",
    "v6_xydata_sqz.dx": "test/v6/xydata_sqz.dx",
    "blood_01.dx": "blood/blood_01.dx",
}


def affn_values(path: str) -> np.ndarray:
    text = open(path).read()
    data = text.split("##XYDATA=")[1].split("\n", 1)[1].split("##")[0]
    vals = []
    for line in data.splitlines():
        vals.extend(float(t) for t in line.split()[1:])
    return np.array(vals)


def main():
    os.makedirs(OUT, exist_ok=True)
    for dst, src in FILES.items():
        with open(os.path.join(REF, src), "rb") as f, \
                gzip.GzipFile(os.path.join(OUT, dst + ".gz"), "wb", 9, mtime=0) as g:
            shutil.copyfileobj(f, g)
    y = affn_values(os.path.join(REF, "test/v6/xydata_affn.dx"))
    assert y.size == 131072 and np.all(y == np.round(y))
    np.savez_compressed(os.path.join(OUT, "blood_01_affn.npz"), intensities=y.astype(np.int64))


if __name__ == "__main__":
    main()
