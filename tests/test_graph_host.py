"""Host side of the schedule processors vs the reference's outputs (decomposition.json)."""
import random
import re

import numpy as np
import pytest

from conftest import golden_json

NAMES = ["0", "1", "2", "3", "4", "5", "er64"]


def _base(pkg, name, ent):
    if name == "er64":
        return [[tuple(e) for e in ent["base"][0]]]
    return pkg.select_graph(int(name))


def test_select_graph_matches_reference_data(pkg):
    dec = golden_json("decomposition")
    for g in range(6):
        assert [[list(e) for e in m] for m in pkg.select_graph(g)] == dec[str(g)]["base"]
        assert pkg.GRAPH_SIZES[g] == dec[str(g)]["size"]


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("seed", ["0", "1", "2"])
def test_decomposition_and_partner_table(pkg, name, seed):
    ent = golden_json("decomposition")[name]
    random.seed(int(seed))
    gp = pkg.GraphProcessor(_base(pkg, name, ent), 1.0, 0, ent["size"], 4, False)
    ref = ent["seeds"][seed]
    assert [[list(map(int, e)) for e in sg] for sg in gp.subGraphs] == ref["subgraphs"]
    assert gp.neighbors_info == ref["neighbors_info"]
    diag = np.diag(sum(gp.L_matrices)).tolist()
    assert diag == ref["laplacian_sum_diag"]


@pytest.mark.parametrize("name", NAMES)
def test_fixed_alpha(pkg, name):
    ent = golden_json("decomposition")[name]
    random.seed(0)
    gp = pkg.GraphProcessor(_base(pkg, name, ent), 1.0, 0, ent["size"], 4, False)
    fp = object.__new__(pkg.FixedProcessor)          # getAlpha needs no GPU
    fp.size, fp.L_matrices = gp.size, gp.L_matrices
    assert fp.getAlpha() == ent["seeds"]["0"]["alpha"]
    if ent["given_alpha"] is not None:
        gg = pkg.GraphProcessor(_base(pkg, name, ent), 1.0, 0, ent["size"], 4, True)
        fp.L_matrices = gg.L_matrices
        assert fp.getAlpha() == ent["given_alpha"]
        assert gg.neighbors_info == ent["given_neighbors_info"]


def test_laplacians_are_laplacians(pkg):
    gp = pkg.GraphProcessor(pkg.select_graph(2), 1.0, 0, 16, 4, True)
    for L, sg in zip(gp.L_matrices, gp.subGraphs):
        assert L.shape == (16, 16) and (L == L.T).all() and (L.sum(axis=1) == 0).all()
        assert int(np.trace(L)) == 2 * len(sg)


def test_invalid_matching_exits_like_reference(pkg, capsys):
    with pytest.raises(SystemExit):
        pkg.GraphProcessor([[(0, 1), (1, 2)]], 1.0, 0, 3, 4, True)
    assert re.search(r"invalide graph! graph: 1", capsys.readouterr().out)


def test_invalid_double_edge_exits(pkg, capsys):
    gp = object.__new__(pkg.GraphProcessor)
    gp.size = 4
    with pytest.raises(SystemExit):
        gp.decomposition([(0, 1), (1, 0)])
    assert "Double edge" in capsys.readouterr().out
