"""The reference-shaped class API (skillshot_learning_amd.game) driven exactly
like the reference and compared with the reference fixtures, on both
libskillshot backends: the CPU backend (device="cpu", csrc/sk_host.cpp; runs
in the CPU suite) and the GPU engine (device="cuda", marked gpu)."""
import contextlib
import io
import math

import numpy as np
import pytest
import torch

import golden_replay as gr

class _Game:
    """the game module with SkillshotGame bound to one backend"""

    def __init__(self, mod, device):
        self._m, self.device = mod, device
        self.FEATURE_KEYS = mod.FEATURE_KEYS

    def SkillshotGame(self, random_positions=False):
        return self._m.SkillshotGame(random_positions=random_positions, device=self.device)


@pytest.fixture(scope="module", params=["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def game_mod(request):
    if request.param == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    from skillshot_learning_amd import game
    return _Game(game, request.param)


def _set(g, d, e, t):
    for k, pl in enumerate((g.player1, g.player2)):
        pl.pos = d["pos"][e, t, k].tolist()
        pl.rotation = float(d["rot"][e, t, k])
        q = pl.projectile
        q.pos = d["qpos"][e, t, k].tolist()
        q.rotation = float(d["qrot"][e, t, k])
        q.cooldown_current = int(d["qcd"][e, t, k])
        q.age = int(d["qage"][e, t, k])
        q.valid = bool(d["qvalid"][e, t, k])
    g.ticks = int(d["ticks"][e, t])
    g.game_live = bool(d["live"][e, t])
    g.winner_id = int(d["winner"][e, t])


def _check(g, d, e, t):
    for k, pl in enumerate((g.player1, g.player2)):
        assert pl.pos == d["pos"][e, t, k].tolist(), (e, t, k)
        assert pl.rotation == float(d["rot"][e, t, k]), (e, t, k)
        q = pl.projectile
        assert q.pos == d["qpos"][e, t, k].tolist()
        assert q.rotation == float(d["qrot"][e, t, k])
        assert (q.cooldown_current, q.age, int(q.valid)) == (int(d["qcd"][e, t, k]), int(d["qage"][e, t, k]),
                                                             int(d["qvalid"][e, t, k]))
    assert (g.ticks, int(g.game_live), g.winner_id) == (int(d["ticks"][e, t]), int(d["live"][e, t]),
                                                         int(d["winner"][e, t]))


def test_raw_protocol_through_class_api(game_mod):
    d = gr.load("raw")
    for e in range(d["pos"].shape[0]):
        g = game_mod.SkillshotGame()
        _set(g, d, e, 0)
        out = io.StringIO()
        with contextlib.redirect_stdout(out):
            for t in range(int(d["n_steps"][e])):
                for pid in (1, 2):
                    pl = g.get_player_by_id(pid)
                    pl.move_direction_float(float(d["actions"][e, t, pid - 1, 0]))
                    pl.move_look_float(float(d["actions"][e, t, pid - 1, 1]))
                    if d["shoot"][e, t, pid - 1]:
                        pl.move_shoot_projectile()
                g.game_tick()
                if t % 7 == 0 or t + 1 == int(d["n_steps"][e]):
                    _check(g, d, e, t + 1)
        if d["winner"][e, -1]:
            assert out.getvalue().strip() == f"Player {int(d['winner'][e, -1])} loss"


def test_learner_protocol_and_get_state(game_mod):
    d = gr.load("int_start_limit200")
    for e in range(3):
        g = game_mod.SkillshotGame()
        _set(g, d, e, 0)
        with contextlib.redirect_stdout(io.StringIO()):
            for t in range(int(d["n_steps"][e])):
                for pid in (1, 2):  # SkillshotLearner.do_actions :206-213
                    a = d["actions"][e, t, pid - 1]
                    g.get_player_by_id(pid).move_direction_float(float(a[0]))
                    g.get_player_by_id(pid).move_look_float(float(a[1]))
                    g.get_player_by_id(pid).move_shoot_projectile()
                g.game_tick()
        _check(g, d, e, int(d["n_steps"][e]))


def test_get_state_and_board(game_mod):
    d = gr.load("boards")
    keys = game_mod.FEATURE_KEYS
    g = game_mod.SkillshotGame()
    for k in range(d["pos"].shape[0]):
        for p, pl in enumerate((g.player1, g.player2)):
            pl.pos = d["pos"][k, p].tolist()
            pl.rotation = float(d["rot"][k, p])
            pl.projectile.pos = d["qpos"][k, p].tolist()
            pl.projectile.rotation = float(d["qrot"][k, p])
            pl.projectile.cooldown_current = int(d["qcd"][k, p])
            pl.projectile.age = int(d["qage"][k, p])
            pl.projectile.valid = bool(d["qvalid"][k, p])
        g.ticks = int(d["ticks"][k])
        g.game_live = bool(d["live"][k])
        g.winner_id = int(d["winner"][k])
        st = g.get_state()
        assert [int(st["game_live"]), st["ticks"], st["game_winner"]] == d["general"][k].tolist()
        for p, pid in ((0, 1), (1, 2)):
            for j, key in enumerate(keys):
                want = d["features"][k, p, j]
                assert abs(float(st[pid][key]) - want) <= 1e-12 * max(1.0, abs(want)), (k, pid, key)
        assert np.array_equal(g.get_board(), d["board"][k])
        # static helpers are the reference's own formulas
        for pid in (1, 2):
            pl, opp = g.get_player_by_id(pid), g.get_player_by_id(3 - pid)
            assert g.check_future_collision(pl.projectile, opp) == bool(st[pid]["projectile_future_collision_opponent"])
            gd = pl.get_gradient_dir()
            assert math.isclose(g.get_dist_line_point(gd["gradient"], pl.pos, opp.pos),
                                st[pid]["player_path_dist_opponent"], rel_tol=1e-12, abs_tol=1e-9)


def test_reset_and_errors(game_mod):
    np.random.seed(3)
    g = game_mod.SkillshotGame(random_positions=True)
    np.random.seed(3)
    want = np.random.randint(25, 225, (2, 2))
    assert g.player1.pos == want[0].tolist() and g.player2.pos == want[1].tolist()
    g.game_reset()
    assert g.player1.pos == [50, 50] and g.player2.pos == [200, 200]
    assert g.get_player_by_id(3) is None
    with pytest.raises(ValueError):
        g.player1.move_direction_float(float("nan"))
    g.player1.pos[0] = 60  # write-through list
    assert g.player1.pos == [60, 50]
    g.player1.move_look_left()
    assert g.player1.rotation == 0.25
    g.player1.move_forwards()
    assert g.player1.pos == [int(round(60 - math.sin(0.25) * 3)), int(round(50 - math.cos(0.25) * 3))]
    x, y = g.player1.pos
    g.player2.projectile.pos = [x + 1, y + 3]  # corners (x+4|x+1, y+3|y) inside P1's 5x5 box
    g.player2.projectile.valid = True
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        g.check_collision()
    assert out.getvalue().strip() == "Player 1 loss" and g.winner_id == 1 and not g.game_live
