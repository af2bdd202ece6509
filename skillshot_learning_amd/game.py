"""Reference-shaped class API over libskillshot: SkillshotGame, Player,
Projectile with the constructors, attributes and methods of
SkillshotGame.py:8-169, Player.py:8-100 and Projectile.py:4-64.

Each SkillshotGame is a one-game VecSkillshotGame: by default on
libskillshot's CPU backend (device="cpu", csrc/sk_host.cpp: one C call per
method, no device round trip), or on the GPU (device="cuda": every mutating
method one launch of the batched kernels with N=1).  Attribute reads come
from a snapshot of the state planes refreshed after mutations.  Pure
helpers the reference computes from attributes alone (get_gradient_dir,
check_pos_valid, the static distance helpers, check_future_collision,
get_board) are evaluated on the host exactly as the reference writes them.

Random starts keep the reference's numpy global RNG draw
(np.random.randint(25, 225, (2, 2)), SkillshotGame.py:15) so np.random.seed
keeps its meaning.
"""
import math

import numpy as np
import torch

from . import _capi
from .vec_env import FEATURE_KEYS, VecSkillshotGame

# get_state value types (SkillshotGame.py:145-163): Python ints, bools and floats
_INTS = {"player_x_dir", "player_pos_x", "player_pos_y", "projectile_cooldown", "projectile_x_dir",
         "projectile_pos_x", "projectile_pos_y", "projectile_age"}
_BOOLS = {"projectile_valid", "projectile_future_collision_opponent"}
_CASTS = tuple(int if k in _INTS else (bool if k in _BOOLS else float) for k in FEATURE_KEYS)

_PLAYER_SHAPE = [[0, 0, 0, 0, 0], [0, 1, 1, 1, 0], [0, 1, 1, 1, 0], [0, 1, 1, 1, 0], [0, 0, 0, 0, 0]]
_PROJECTILE_SHAPE = [[1, 0, 1], [0, 1, 0], [1, 0, 1]]


class _WriteThroughList(list):
    """A [x, y] list whose item assignment writes the game state."""

    def __init__(self, values, setter):
        super().__init__(values)
        self._setter = setter

    def __setitem__(self, idx, value):
        super().__setitem__(idx, value)
        self._setter(list(self))


def _gradient_dir(rotation, pos):
    # Player.get_gradient_dir (Player.py:91-100) == Projectile.get_gradient_dir (Projectile.py:55-64)
    gradient = math.tan(-rotation + math.pi / 2)
    x_dir = 1 if -math.sin(rotation) >= 0 else -1
    y_intercept = pos[1] - gradient * pos[0]
    return dict(gradient=gradient, x_dir=x_dir, y_intercept=y_intercept)


def _nan_check(x):
    if isinstance(x, float) and math.isnan(x):
        raise ValueError("cannot convert float NaN to integer")  # int(round(nan)) in the reference


def _trig_check(rotation):
    """math.sin/cos of the rotation raise in the reference before any move."""
    if math.isinf(rotation):
        raise ValueError("math domain error")
    _nan_check(rotation)


def rasterize_board(board, pos, rot, qpos, qvalid):
    """SkillshotGame.get_board (SkillshotGame.py:36-56): players as colour 1/2
    with a direction pixel 3/4, valid projectiles as 3/4, [x, y] indexing."""
    board = np.array(board, copy=True)
    sx, sy = len(_PLAYER_SHAPE[0]), len(_PLAYER_SHAPE)
    for k, (colour, pointer) in enumerate(((1, 3), (2, 4))):
        px_dir = math.floor(-math.sin(rot[k]) * sx / 2 + sx / 2)
        py_dir = math.floor(-math.cos(rot[k]) * sy / 2 + sy / 2)
        for index_y, row in enumerate(_PLAYER_SHAPE):
            for index_x, item in enumerate(row):
                if item != 0:
                    board[index_x + pos[k][0], index_y + pos[k][1]] = colour
                if index_x == px_dir and index_y == py_dir:
                    board[index_x + pos[k][0], index_y + pos[k][1]] = pointer
        if qvalid[k]:
            for index_y, row in enumerate(_PROJECTILE_SHAPE):
                for index_x, item in enumerate(row):
                    if item != 0:
                        board[index_x + qpos[k][0], index_y + qpos[k][1]] = pointer
    return board


class Projectile(object):
    """View of one player's projectile (Projectile.py:4-64)."""
    shape_image = _PROJECTILE_SHAPE
    cooldown_max = 15
    speed_move = 5

    def __init__(self, game, index):
        self._g = game
        self._i = index
        self.board_dim = game.board_size
        self.shape_size = (len(self.shape_image[0]), len(self.shape_image))

    # -- attributes
    @property
    def pos(self):
        s = self._g._snap()
        return _WriteThroughList([int(s["qpos"][0, 2 * self._i]), int(s["qpos"][0, 2 * self._i + 1])],
                                 self.set_position)

    @pos.setter
    def pos(self, value):
        self.set_position(value)

    @property
    def rotation(self):
        return float(self._g._snap()["rot_q"][self._i])

    @rotation.setter
    def rotation(self, value):
        self.set_rotation(value)

    @property
    def cooldown_current(self):
        return int(self._g._snap()["qcdage"][0, 2 * self._i])

    @cooldown_current.setter
    def cooldown_current(self, value):
        self._g._write("qcdage", (0, 2 * self._i), int(value))

    @property
    def age(self):
        return int(self._g._snap()["qcdage"][0, 2 * self._i + 1])

    @age.setter
    def age(self, value):
        self._g._write("qcdage", (0, 2 * self._i + 1), int(value))

    @property
    def valid(self):
        return bool(self._g._flag(self._i))

    @valid.setter
    def valid(self, value):
        self._g._set_flag(self._i, 1 if value else 0)

    # -- methods
    def set_position(self, location):  # Projectile.py:22-24
        loc = list(location)
        self._g._write("qpos", (0, 2 * self._i), int(loc[0]))
        self._g._write("qpos", (0, 2 * self._i + 1), int(loc[1]))

    def set_rotation(self, rotation):  # Projectile.py:26-28
        self._g._write("qrot", (0, self._i), float(rotation))

    def check_pos_valid(self, check_x, check_y):  # Projectile.py:30-36
        return (check_x + self.shape_size[0] <= self.board_dim[0] and check_x >= 0 and
                check_y + self.shape_size[1] <= self.board_dim[1] and check_y >= 0)

    def move_forwards(self):  # Projectile.py:38-47
        _trig_check(self.rotation)
        self._g._projectile_move(self._i + 1, 0)

    def tick(self):  # Projectile.py:49-53
        _trig_check(self.rotation)
        self._g._projectile_move(self._i + 1, 1)

    def get_gradient_dir(self):
        return _gradient_dir(self.rotation, self.pos)


class Player(object):
    """View of one player (Player.py:8-100)."""
    shape_image = _PLAYER_SHAPE
    speed_move = 3
    speed_look = 0.25

    def __init__(self, game, index):
        self._g = game
        self._i = index
        self.id = index + 1
        self.board_dim = game.board_size
        self.shape_size = (len(self.shape_image[0]), len(self.shape_image))
        self.projectile = Projectile(game, index)

    @property
    def pos(self):
        s = self._g._snap()
        return _WriteThroughList([int(s["pos"][0, 2 * self._i]), int(s["pos"][0, 2 * self._i + 1])],
                                 self._set_pos)

    @pos.setter
    def pos(self, value):
        self._set_pos(list(value))

    def _set_pos(self, value):
        self._g._write("pos", (0, 2 * self._i), int(value[0]))
        self._g._write("pos", (0, 2 * self._i + 1), int(value[1]))

    @property
    def rotation(self):
        return float(self._g._snap()["rot_p"][self._i])

    def _rotation_checked(self):
        """the rotation, raising where the reference's math.sin/cos would"""
        r = float(self._g._snap()["rot_p"][self._i])
        if r != r or r in (math.inf, -math.inf):
            _trig_check(r)
        return r

    @rotation.setter
    def rotation(self, value):
        self._g._write("rot", (0, self._i), float(value))

    def move_look_left(self):  # Player.py:27-28
        self._g._move_discrete(self.id, 2)

    def move_look_right(self):  # Player.py:30-31
        self._g._move_discrete(self.id, 3)

    def move_look_float(self, angle):  # Player.py:33-39
        self._g._move_look(self.id, float(angle))

    def move_forwards(self):  # Player.py:41-47
        self._rotation_checked()
        self._g._move_discrete(self.id, 0)

    def move_backwards(self):  # Player.py:49-55
        self._rotation_checked()
        self._g._move_discrete(self.id, 1)

    def move_direction_float(self, speed):  # Player.py:57-68
        speed = float(speed)
        self._rotation_checked()
        if speed != speed:  # int(round(nan)) raises in the reference
            _nan_check(speed)
        self._g._move_direction(self.id, speed)

    def check_pos_valid(self, check_x, check_y):  # Player.py:70-76
        return (check_x + self.shape_size[0] <= self.board_dim[0] and check_x >= 0 and
                check_y + self.shape_size[1] <= self.board_dim[1] and check_y >= 0)

    def move_shoot_projectile(self):  # Player.py:78-89
        self._g._shoot(self.id)

    def get_gradient_dir(self):  # Player.py:91-100
        return _gradient_dir(self.rotation, self.pos)


class SkillshotGame(object):
    """SkillshotGame.py:8-169 over a one-game libskillshot batch (CPU backend or GPU)."""

    def __init__(self, random_positions=False, device="cpu"):
        self.board_size = (250, 250)
        self.board = np.zeros(self.board_size, dtype=int)
        if getattr(self, "_eng", None) is None:
            self._eng = VecSkillshotGame(1, device=device, tick_limit=2 ** 31 - 1, random_positions=False)
            self._bind()
        self._eng.reset(random_positions=False)
        self._dirty()
        if random_positions:
            pos_player1, pos_player2 = np.random.randint(25, 225, (2, 2))  # SkillshotGame.py:15
            self._write("pos", (0, 0), int(pos_player1[0]))
            self._write("pos", (0, 1), int(pos_player1[1]))
            self._write("pos", (0, 2), int(pos_player2[0]))
            self._write("pos", (0, 3), int(pos_player2[1]))
        self.player1 = Player(self, 0)
        self.player2 = Player(self, 1)

    # -- state plumbing
    def _bind(self):
        """the per-method entry points: direct C calls on the CPU backend
        (host pointers, no stream; the state planes are live numpy views, so
        the snapshot never goes stale), the VecSkillshotGame methods on the
        GPU (snapshot refreshed after each mutation)"""
        e = self._eng
        self._cpu = e.is_cpu
        self._cache = None
        if self._cpu:
            L, h = e._L, e._h
            views = {k: getattr(e, k).numpy() for k in ("pos", "rot", "qpos", "qrot", "qcdage", "misc")}
            views["rot_p"] = views["rot"][0]
            views["rot_q"] = views["qrot"][0]
            self._cache = views
            ck = _capi.check  # SK_EINVAL etc. raise here as on the GPU path
            self._move_direction = lambda pid, v: ck(L.sk_player_move_direction(h, pid, None, v, None))
            self._move_look = lambda pid, v: ck(L.sk_player_move_look(h, pid, None, v, None))
            self._move_discrete = lambda pid, k: ck(L.sk_player_move_discrete(h, pid, k, None, None))
            self._shoot = lambda pid: ck(L.sk_player_shoot(h, pid, None, None))
            self._projectile_move = lambda pid, t: ck(L.sk_projectile_move(h, pid, t, None, None))
            self._game_tick_c = lambda: ck(L.sk_game_tick(h, None))
        else:
            def mut(f):
                def g(*a):
                    f(*a)
                    self._cache = None
                return g
            self._move_direction = mut(e.move_direction)
            self._move_look = mut(e.move_look)
            self._move_discrete = mut(e.move_discrete)
            self._shoot = mut(e.shoot)
            self._projectile_move = mut(lambda pid, t: e.projectile_move(pid, tick=bool(t)))
            self._game_tick_c = mut(e.game_tick)

    def _dirty(self):
        if not self._cpu:
            self._cache = None

    def _snap(self):
        if self._cache is None:
            if self._eng.is_cpu:  # the planes are host memory: views, no copies
                d = {k: getattr(self._eng, k).numpy() for k in ("pos", "rot", "qpos", "qrot", "qcdage", "misc")}
            else:
                torch.cuda.current_stream(self._eng.device).synchronize()
                d = {k: getattr(self._eng, k).cpu().numpy() for k in ("pos", "rot", "qpos", "qrot", "qcdage",
                                                                      "misc")}
            d["rot_p"] = d["rot"][0]
            d["rot_q"] = d["qrot"][0]
            self._cache = d
        return self._cache

    def _write(self, plane, idx, value):
        getattr(self._eng, plane)[idx] = value
        self._dirty()

    def _flags(self):
        return int(self._snap()["misc"][0, 1]) & 0xFFFFFFFF

    def _flag(self, byte):
        return (self._flags() >> (8 * byte)) & 0xFF

    def _set_flag(self, byte, value):
        f = self._flags()
        f = (f & ~(0xFF << (8 * byte))) | ((int(value) & 0xFF) << (8 * byte))
        self._write("misc", (0, 1), int(np.uint32(f).view(np.int32)))

    # -- attributes
    @property
    def ticks(self):
        return int(self._snap()["misc"][0, 0])

    @ticks.setter
    def ticks(self, v):
        self._write("misc", (0, 0), int(v))

    @property
    def game_live(self):
        return bool(self._flag(2))

    @game_live.setter
    def game_live(self, v):
        self._set_flag(2, 1 if v else 0)

    @property
    def winner_id(self):
        return int(self._flag(3))

    @winner_id.setter
    def winner_id(self, v):
        self._set_flag(3, int(v))

    # -- methods
    def get_player_by_id(self, player_id):  # SkillshotGame.py:27-34
        if self.player1.id == player_id:
            return self.player1
        elif self.player2.id == player_id:
            return self.player2
        return None

    def get_board(self):  # SkillshotGame.py:36-56 (host rasteriser, visualisation only)
        return rasterize_board(self.board, [p.pos for p in (self.player1, self.player2)],
                               [p.rotation for p in (self.player1, self.player2)],
                               [p.projectile.pos for p in (self.player1, self.player2)],
                               [p.projectile.valid for p in (self.player1, self.player2)])

    def check_collision(self):  # SkillshotGame.py:58-94
        hit = int(self._eng.check_collision().cpu()[0])
        self._dirty()
        if hit:
            print("Player", hit, "loss")

    @staticmethod
    def check_future_collision(projectile, opponent):  # SkillshotGame.py:96-113
        if projectile.valid:
            grad = projectile.get_gradient_dir()
            qpos, opos = projectile.pos, opponent.pos
            for x_bound_projectile in (qpos[0], qpos[0] + projectile.shape_size[0]):
                for x_bound_opponent in (opos[0], opos[0] + opponent.shape_size[0]):
                    if (x_bound_projectile - qpos[0]) * grad.get("x_dir") >= 0:
                        if opos[1] <= grad.get("gradient") * x_bound_opponent + grad.get("y_intercept") <= \
                                opos[1] + opponent.shape_size[1]:
                            return True
        return False

    def game_tick(self):  # SkillshotGame.py:115-122
        was_live = self.game_live
        if was_live:  # Projectile.move_forwards evaluates sin/cos before testing valid
            qr = self._snap()["rot_q"]
            for r in (float(qr[0]), float(qr[1])):
                if r != r or r in (math.inf, -math.inf):
                    _trig_check(r)
        self._game_tick_c()
        if was_live and not self.game_live:
            print("Player", self.winner_id, "loss")

    @staticmethod
    def get_dist_line_point(line_gradient, line_point, comparison_point):  # SkillshotGame.py:124-130
        c = (line_point[1] - line_gradient * line_point[0])
        return abs(line_gradient * comparison_point[0] - comparison_point[1] + c) / math.sqrt(line_gradient ** 2 + 1)

    @staticmethod
    def get_dist_point_point(point1, point2):  # SkillshotGame.py:132-134
        return ((point1[0] - point2[0]) ** 2 + (point1[1] - point2[1]) ** 2) ** 0.5

    def get_state(self):  # SkillshotGame.py:136-166, numerics from sk_env_features
        if self._cpu:
            fb = getattr(self, "_featbuf", None)
            if fb is None:
                fb = self._featbuf = torch.empty((1, 2, 18), dtype=torch.float64)
                self._featnp = fb.numpy()
            self._eng.features(out=fb)
            f = self._featnp[0].tolist()
        else:
            f = self._eng.features().cpu().numpy()[0].tolist()
        feature_dict = dict(game_live=self.game_live, ticks=self.ticks, game_winner=self.winner_id)
        casts = _CASTS
        for p, pid in ((0, 1), (1, 2)):
            row = f[p]
            feature_dict[pid] = {key: casts[k](row[k]) for k, key in enumerate(FEATURE_KEYS)}
        return feature_dict

    def game_reset(self, random_positions=False):  # SkillshotGame.py:168-169
        self.__init__(random_positions=random_positions)
