"""F4 row: get_board rasteriser and the oracle's get_state numerics against
reference fixtures (tests/golden/boards.npz), on CPU."""
import numpy as np

import golden_replay as gr
from skillshot_learning_amd.game import rasterize_board


def test_rasterize_board_matches_reference():
    d = gr.load("boards")
    for k in range(d["board"].shape[0]):
        got = rasterize_board(np.zeros((250, 250), dtype=int), d["pos"][k].tolist(), d["rot"][k].tolist(),
                              d["qpos"][k].tolist(), d["qvalid"][k].tolist())
        assert np.array_equal(got, d["board"][k]), k


def test_oracle_features_match_reference_get_state(oracle_mod):
    d = gr.load("boards")
    n = d["pos"].shape[0]
    s = oracle_mod.OracleState(n)
    flags = oracle_mod.pack_flags(d["qvalid"], d["live"], d["winner"])
    s.load(dict(pos=d["pos"].reshape(n, 4), rot=d["rot"], qpos=d["qpos"].reshape(n, 4), qrot=d["qrot"],
                qcdage=np.stack([d["qcd"][:, 0], d["qage"][:, 0], d["qcd"][:, 1], d["qage"][:, 1]], -1),
                misc=np.stack([d["ticks"], flags], -1)))
    f = s.features()
    w = d["features"]
    assert np.array_equal(f[..., 17], w[..., 17])
    assert (np.abs(f - w) / np.maximum(1, np.abs(w))).max() <= 1e-12
