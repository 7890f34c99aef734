"""configs[0] golden: the reference ``chromatin.py`` on its own ``example/example.vcf`` (10 SNVs on
chr1 up to 11.08 Mb; copied to tests/golden/example.vcf as an input fixture) at the default
``--maxshift 800``, over a seeded synthetic 12 Mb chr1 (hg19 is not available offline), with
the seeded Beluga weights and the pyfasta/h5py stubs (make_golden.py).

Run from the repo root (needs /root/reference; never read at test time):
    python tests/golden/make_golden_example.py

Writes tests/golden/example_chromatin.npz: per shift, every row of diff/ref/alt at every 4th
feature, plus float64 row sums over all 2002 features; stdout lines and snps_hg19.vcf.
The genome is regenerated at test time by ``genome()`` (same seed).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
GOLD = os.path.join(REPO, "tests", "golden")
STUBS = os.path.join(GOLD, "stubs")
SHIFTS = [0, -200, -400, -600, -800, 200, 400, 600, 800]     # chromatin.py:243 at --maxshift 800


def genome() -> dict:
    sys.path.insert(0, REPO)
    from expecto_amd import synthetic
    return synthetic.genome_bytes(n_contigs=1, contig_len=12_000_000, seed=11)


def main():
    import torch
    sys.path.insert(0, REPO)
    from expecto_amd import synthetic
    from oracle import weights as oweights
    work = tempfile.mkdtemp(prefix="expecto_golden_example_")
    os.makedirs(os.path.join(work, "resources"))
    synthetic.write_fasta(os.path.join(work, "resources", "hg19.fa"), genome())
    torch.save(oweights.seeded_state_dict(0), os.path.join(work, "resources", "deepsea.beluga.pth"))
    shutil.copy(os.path.join(GOLD, "example.vcf"), os.path.join(work, "example.vcf"))
    env = dict(os.environ, PYTHONPATH=STUBS + ":" + REF, OMP_NUM_THREADS="8")
    out = subprocess.run([sys.executable, os.path.join(REF, "chromatin.py"), "example.vcf", "--output_dir", "out"],
                         cwd=work, env=env, capture_output=True, text=True, check=True)
    res = {}
    for s in SHIFTS:
        with np.load(os.path.join(work, "out", f"snps.shift_{s}.diff.h5.npz")) as z:
            for k in ("diff", "ref", "alt"):
                res[f"{k}_{s}"] = z[k][:, ::4]
                res[f"{k}_sum_{s}"] = z[k].astype(np.float64).sum(1)
                res[f"{k}_shape_{s}"] = np.array(z[k].shape)
    res["stdout"] = np.array([l for l in out.stdout.splitlines() if l.startswith("Number of")])
    res["snps_hg19"] = np.array(open(os.path.join(work, "out", "snps_hg19.vcf")).read())
    np.savez_compressed(os.path.join(GOLD, "example_chromatin.npz"), **res)
    shutil.rmtree(work)
    print("configs[0] golden written:", out.stdout[-300:])


if __name__ == "__main__":
    main()
