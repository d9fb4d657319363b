"""GPU: ontologies read from OWL functional syntax (loader + normalizer)
classified by the HIP engine, checked against the CPU oracle; the CLI writes the
``X|B`` result file and the ELK-style diff of it against the oracle's finds nothing."""
import glob
import os

import numpy as np
import pytest

from distel_amd import cli, engine, generators, owl
from distel_amd.result import ResultNode, diff_results, read_saxioms

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "owl")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "*.ofn"))), ids=os.path.basename)
def test_owl_kat_gpu(path, oracle_lib):
    with pytest.warns(UserWarning):
        ax = owl.load_functional(path)
    eng, st = engine.classify(ax)
    o = oracle_lib.saturate(ax, 0)
    for g, c in zip(eng.facts() + eng.links(), o.facts() + o.links()):
        assert np.array_equal(g, c)
    eng.close()


def test_generated_owl_file_gpu(tmp_path, oracle_lib):
    """G1 (chains, CR4, definitions) written as OWL, read back (isNormalized=true), and
    classified: same closure as the IR it was written from; the CLI's X|B file diffs clean."""
    ax = generators.workload("g1", scale=0.05)
    path = tmp_path / "g1.ofn"
    owl.write_functional(owl.from_axioms(ax), str(path))
    bx = owl.load_functional(str(path), normalized=True)
    assert bx.counts() == ax.counts()
    eng, st = engine.classify(bx)
    o = oracle_lib.saturate(ax, 0)
    assert st["derived"] == o.stats()["derived"]
    eng.close()
    out = tmp_path / "res.txt"
    assert cli.main(["classify", str(path), "--normalized", "--out", str(out), "--names"]) == 0
    ox, oa = oracle_lib.saturate(bx, 0).facts()
    ref = tmp_path / "ref.txt"
    ResultNode(bx, ox, oa, distel_compat=False).write_saxioms(str(ref), use_names=True)
    misses, rep = diff_results(read_saxioms(str(ref)), read_saxioms(str(out)))
    assert misses == 0, rep[:5]
    out2 = tmp_path / "res2.txt"
    assert cli.main(["classify", str(path), "--normalized", "--out", str(out2), "--names", "--parts", "3"]) == 0
    assert read_saxioms(str(out2)) == read_saxioms(str(out))
