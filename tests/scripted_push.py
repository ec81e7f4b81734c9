"""A scripted policy that works the cube (test infrastructure): per env a randomised approach that
brings the tool bar and the hand down beside the cube and pushes it across the table (the task of
push.py:30-47), so Bullet's persistent manifolds of the robot / cube pairs see merges, appends,
area replacements and both removals of refreshContactPoints -- which the random policy, whose arm
rarely meets the cube, does not exercise.  EE control (Push / PickAndPlace, panda.py:226-246: the
action moves the IK target by 0.05 a), computed from the observation (obs 0:3 the EE; the cube at
obs 6:9 in Push, 7:10 in PickAndPlace, whose obs carries the fingers' width at 6).  The script
restarts every 50 steps (the TimeLimit's episode).

Per env, drawn once from a seeded generator: the push direction, a lateral offset of the contact
point (bar centred or on the cube's edge, so it turns), the push height (bar on the cube's face
or pressing its top edge) and the approach length; small per-step noise keeps the contacts moving.
"""
import numpy as np

STAND_OFF = 0.075       # pre-push point behind the cube centre (m)


class ScriptedPush:
    def __init__(self, n: int, seed: int = 0, obj_col: int = 6):
        self.obj_col = obj_col
        rng = np.random.default_rng(seed)
        th = rng.uniform(-np.pi, np.pi, n)
        self.d = np.stack([np.cos(th), np.sin(th), np.zeros(n)], axis=1)            # push direction
        self.side = np.stack([-np.sin(th), np.cos(th), np.zeros(n)], axis=1)
        self.offset = rng.uniform(-0.025, 0.025, n)                                  # lateral contact offset
        self.height = rng.uniform(0.036, 0.06, n)                                    # EE height while pushing
        self.t_down = rng.integers(5, 9, n)                                          # steps to the pre-push point
        self.rng = np.random.default_rng(seed + 1)
        self.pre = None

    def __call__(self, obs: np.ndarray, t: int) -> np.ndarray:
        t = t % 50
        ee, cube = obs[:, 0:3].astype(np.float64), obs[:, self.obj_col:self.obj_col + 3].astype(np.float64)
        if self.pre is None or t == 0:
            self.pre = cube - STAND_OFF * self.d + self.offset[:, None] * self.side
        tgt = self.pre.copy()
        tgt[:, 2] = 0.12                                        # above the cube first
        down = (t >= self.t_down)[:, None]
        low = self.pre.copy()
        low[:, 2] = self.height
        tgt = np.where(down, low, tgt)
        push = (t >= self.t_down + 4)[:, None]
        through = cube + 0.12 * self.d + self.offset[:, None] * self.side
        through[:, 2] = self.height
        tgt = np.where(push, through, tgt)
        a = (tgt - ee) / 0.05 + self.rng.normal(0.0, 0.15, ee.shape)
        return np.clip(a, -1.0, 1.0).astype(np.float32)
