"""A scripted policy that works the cube (test infrastructure): per env a randomised approach that
brings the tool bar and the hand down beside the cube and pushes it across the table (the task of
push.py:30-47), so Bullet's persistent manifolds of the robot / cube pairs see merges, appends,
area replacements and both removals of refreshContactPoints -- which the random policy, whose arm
rarely meets the cube, does not exercise.  EE control (Push / PickAndPlace, panda.py:226-246: the
action moves the IK target by 0.05 a), computed from the observation (obs 0:3 the EE; the cube at
obs 6:9 in Push, 7:10 in PickAndPlace, whose obs carries the fingers' width at 6).  The script
restarts every 50 steps (the TimeLimit's episode).

Per env, drawn once from a seeded generator: the push direction (towards the centre of the cubes'
spawn region, +-45 deg, so the cube stays on the table), a lateral offset of the contact point (bar
centred or on the cube's edge, so it turns), the push height (the bar on the cube's upper face half,
which pushes instead of wedging under it) and the approach length; small per-step noise keeps the
contacts moving.
"""
import numpy as np

STAND_OFF = 0.075       # pre-push point behind the cube centre (m)


class ScriptedPush:
    def __init__(self, n: int, seed: int = 0, obj_col: int = 6, height=(0.056, 0.072), rough: bool = False):
        """height: the EE height range while pushing -- the tool bar's underside sits 0.0416 below
        the EE, so the default keeps it just off the table (the bar sliding on the table under
        load is the table-drive regime, test_reach_with_table_contacts); lower bounds press it on."""
        self.obj_col = obj_col
        # rough: any direction, the full action range, the end point chasing the cube -- the arm
        # shoves and wedges the cube (more robot points at once; cubes can leave the table)
        self.rough = rough
        rng = np.random.default_rng(seed)
        self.turn = rng.uniform(-np.pi / 4, np.pi / 4, n)    # push direction: towards the spawn region's centre +- 45 deg
        self.offset = rng.uniform(-0.025, 0.025, n)                                  # lateral contact offset
        self.height = rng.uniform(height[0], height[1], n)                           # EE height while pushing
        self.t_down = rng.integers(5, 9, n)                                          # steps to the pre-push point
        self.rng = np.random.default_rng(seed + 1)
        self.pre = None

    def __call__(self, obs: np.ndarray, t: int) -> np.ndarray:
        t = t % 50
        ee, cube = obs[:, 0:3].astype(np.float64), obs[:, self.obj_col:self.obj_col + 3].astype(np.float64)
        if self.pre is None or t == 0:
            th = np.arctan2(-cube[:, 1], -cube[:, 0]) + (4.0 * self.turn if self.rough else self.turn)
            self.d = np.stack([np.cos(th), np.sin(th), np.zeros_like(th)], axis=1)
            self.side = np.stack([-np.sin(th), np.cos(th), np.zeros_like(th)], axis=1)
            self.pre = cube - STAND_OFF * self.d + self.offset[:, None] * self.side
            # the end of the push, fixed at the start (chasing the cube would shove it off the table:
            # a cube falling past the edge is test_cube_at_the_table_side_wall_and_edge's case, with
            # its own bar -- here the manifold branches of a cube pushed across the table top)
            self.end = cube + 0.12 * self.d + self.offset[:, None] * self.side
            # and the cube kept on the table's interior (table x in [-0.85, 0.25], |y| <= 0.35, less the
            # cube and a margin): where the push would cross an edge it goes the other way
            out = (self.end[:, 0] > 0.15) | (self.end[:, 0] < -0.75) | (np.abs(self.end[:, 1]) > 0.25)
            if out.any():
                self.d[out] *= -1.0
                self.side[out] *= -1.0
                self.pre[out] = cube[out] - STAND_OFF * self.d[out] + self.offset[out, None] * self.side[out]
                self.end[out] = cube[out] + 0.12 * self.d[out] + self.offset[out, None] * self.side[out]
        tgt = self.pre.copy()
        tgt[:, 2] = 0.12                                        # above the cube first
        down = (t >= self.t_down)[:, None]
        low = self.pre.copy()
        low[:, 2] = self.height
        tgt = np.where(down, low, tgt)
        push = (t >= self.t_down + 4)[:, None]
        through = (cube + 0.12 * self.d + self.offset[:, None] * self.side) if self.rough else self.end.copy()
        through[:, 2] = self.height
        tgt = np.where(push, through, tgt)
        a = (tgt - ee) / 0.05 + self.rng.normal(0.0, 0.15, ee.shape)
        # at most 0.6 of the action range while low: the arm pushes the cube instead of kicking it
        # off the table (see above)
        lim = np.where(down & (not self.rough), 0.6, 1.0)
        return np.clip(a, -lim, lim).astype(np.float32)
