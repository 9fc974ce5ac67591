"""CPU: the LSVC reference-tree helpers (models.py:683-728, 923-949) and the layer schedule the
tree GOP codes."""
import pytest

from fastvideocodec_amd.tree_gop import coding_layers, generate_graph, graph_from_batch, refidx_from_graph


@pytest.mark.parametrize("kind", ["default", "onehop", "2layers", "3layers", "4layers", "5layers"])
def test_graph_consistency(kind):
    g, layers, parents = generate_graph(kind)
    for p, kids in g.items():
        for k in kids:
            assert parents[k] == p
    flat = [t for layer in layers for t in layer]
    assert sorted(flat) == sorted(parents)
    seen = {0}
    for layer in layers:  # every frame's parent is coded in an earlier layer
        assert all(parents[t] in seen for t in layer)
        seen.update(layer)


def test_graph_from_batch_and_refidx():
    # models.py:923-940 size classes
    assert graph_from_batch(2)[1] == [[1, 2]]
    assert graph_from_batch(6)[1] == [[1, 4], [2, 3, 5, 6]]
    assert graph_from_batch(11)[1][0] == [1, 8]
    assert len(graph_from_batch(30)[1]) == 4
    with pytest.raises(ValueError):
        graph_from_batch(31)
    g, _, _ = graph_from_batch(6)
    assert refidx_from_graph(g, 6) == [0, 1, 1, 0, 4, 4]
    g, _, _ = graph_from_batch(11)
    assert refidx_from_graph(g, 11) == [0, 1, 2, 2, 1, 5, 5, 0, 8, 9, 9]


def test_coding_layers_gop12():
    lay = coding_layers(11)
    assert [[t for t, _ in l] for l in lay] == [[1, 8], [2, 5, 9], [3, 4, 6, 7, 10, 11]]
    assert dict(p for l in lay for p in l) == {1: 0, 8: 0, 2: 1, 5: 1, 9: 8, 3: 2, 4: 2, 6: 5, 7: 5, 10: 9, 11: 9}
    assert [[t for t, _ in l] for l in coding_layers(5, isLinear=True)] == [[1], [2], [3], [4], [5]]


def _golden():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "tree_graphs.json")) as f:
        return json.load(f)


def _ints(d):
    return {int(k): v for k, v in d.items()}


def test_graphs_vs_reference_fixture():
    """Pinned to the reference's own helpers (tests/golden/gen_tree_golden.py ran models.py's
    generate_graph / graph_from_batch / refidx_from_graph): every graph type, every batch size
    1..30 in the three modes, and the failure past 30 frames."""
    gold = _golden()
    for kind, e in gold["generate_graph"].items():
        g, layers, parents = generate_graph(kind)
        assert g == _ints(e["g"]) and layers == e["layers"] and parents == _ints(e["parents"]), kind
    for key, e in gold["graph_from_batch"].items():
        bs = int(key.split("-")[0])
        lin, one = "-L" in key, "-O" in key
        g, layers, parents = graph_from_batch(bs, isLinear=lin, isOnehop=one)
        assert layers == e["layers"] and parents == _ints(e["parents"]), key
        assert refidx_from_graph(g, bs) == gold["refidx_from_graph"][key], key
    assert gold["graph_from_batch_31"] != "returned"
    with pytest.raises(ValueError):
        graph_from_batch(31)


def test_binary_tree_extension():
    """binary_tree_graph reproduces the reference's 2..5-layer tables and extends them to the
    62-frame tree that coding_layers(extend=True) uses past 30 P-frames (configs[3]'s GOP-32)."""
    from fastvideocodec_amd.tree_gop import binary_tree_graph
    for depth, kind in ((2, "2layers"), (3, "3layers"), (4, "4layers"), (5, "5layers")):
        assert binary_tree_graph(depth) == generate_graph(kind)
    lay = coding_layers(31, extend=True)
    assert [len(l) for l in lay] == [1, 2, 4, 8, 16]
    par = dict(p for l in lay for p in l)
    assert sorted(par) == list(range(1, 32))
    seen = {0}
    for l in lay:
        assert all(p in seen for _, p in l)
        seen.update(t for t, _ in l)
    with pytest.raises(ValueError):
        coding_layers(31)
