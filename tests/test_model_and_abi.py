"""Model tables (URDF -> Bullet multibody) and the C-ABI boundary, on CPU (no GPU calls)."""
import ctypes as C
import math
import os
import re
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from panda_gym_amd import abi
from panda_gym_amd.model import bullet_quicksort_equal_keys, forward_kinematics, load_model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_link_order_matches_reference_indices():
    """custom_0 links 0-6 panda_link1..7, 9 panda_ee, 11 panda_rightfinger (ee_link, panda.py:68)."""
    m = load_model("panda_custom0")
    assert m.link_names[:7] == [f"panda_link{i}" for i in range(1, 8)]
    assert m.link_names[9] == "panda_ee" and m.link_names[11] == "panda_rightfinger"
    assert m.n_dofs == 7 and all(t == 4 for t in m.jtype[7:])


def test_neutral_ee_position():
    """EE = COM of panda_rightfinger at the neutral pose (panda.py:67), base (-0.6, 0, 0)."""
    m = load_model("panda_custom0")
    fk = forward_kinematics(m, [0, -0.3, 0, -2.2, 0, 2.0, math.pi / 4], base_pos=(-0.6, 0, 0))
    assert np.allclose(fk["C"][11], [-0.11845, 0.01, 0.4375], atol=1e-4)


def test_inertia_is_bullet_aabb_rule():
    """No URDF_USE_INERTIA_FROM_FILE: inertia from the collision AABB, not the URDF <inertia> 0.1."""
    m = load_model("panda_custom0")
    assert all(abs(I[0] - 0.1) > 1e-3 for I, ms in zip(m.inertia, m.mass) if ms > 0)
    # finger links have mass but no collision: empty-compound AABB (2 * margin)
    assert 0 < m.inertia[11][0] < 1e-6


def test_quicksort_permutation_equal_keys():
    assert bullet_quicksort_equal_keys([0, 1]) == [1, 0]
    p = bullet_quicksort_equal_keys(list(range(14)))
    assert sorted(p) == list(range(14))


def test_row_header_matches_model():
    m = load_model("panda_custom0")
    kinds, dofs = m.row_table()
    hdr = open(os.path.join(ROOT, "panda-gym_amd", "csrc", "pgx_rows.h")).read()
    codes = [int(x) for x in re.search(r"\{([0-9, ]+)\}", hdr).group(1).split(",")]
    assert codes == [int(k) << 4 | int(d) for k, d in zip(kinds, dofs)]


def _declared_functions():
    hdr = open(os.path.join(ROOT, "include", "pgx.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\*?\s+\*?(pgx_[a-z_0-9]+)\s*\(", hdr, re.M)))


def test_libpgx_exports_every_declared_symbol():
    from panda_gym_amd import _native

    lib = _native.load()
    decl = _declared_functions()
    assert len(decl) >= 14
    for name in decl:
        assert hasattr(lib, name), name
    assert set(decl) == set(_native.EXPORTS)
    assert lib.pgx_version().startswith(b"pgx")


def test_host_only_calls_without_gpu():
    from panda_gym_amd import _native

    lib = _native.load()
    cfg = abi.make_config(abi.EnvSpec(), 8, abi.make_model(load_model("panda_custom0")), abi.default_sim_params())
    assert lib.pgx_obs_dim(C.byref(cfg)) == 6 and lib.pgx_action_dim(C.byref(cfg)) == 3
    cfg.task = 7                                                 # Slide/Flip/Stack: out of scope
    h = C.c_void_p()
    assert lib.pgx_create(C.byref(cfg), 0, C.byref(h)) < 0      # unsupported task fails loudly
    assert b"task" in lib.pgx_last_error()
    cfg.task, cfg.contacts = abi.TASK_PUSH, 0
    assert lib.pgx_create(C.byref(cfg), 0, C.byref(h)) < 0      # an object needs the contact solver
    assert b"contacts" in lib.pgx_last_error()
    cfg.contacts, cfg.lanes_per_env = abi.CONTACTS_FULL, 1   # the full manifold budget: 16 lanes only
    assert lib.pgx_create(C.byref(cfg), 0, C.byref(h)) == -3
    assert b"16-lane" in lib.pgx_last_error()
    cfg.contacts = 3
    assert lib.pgx_create(C.byref(cfg), 0, C.byref(h)) < 0
    assert lib.pgx_step(None, None, None, None) < 0


def test_compiled_default_model_is_current():
    """The constant block the kernels are compiled with (pgx_default_model.h) is the one pgx_create
    folds today for the default parameters; other parameters are refused before any HIP call."""
    from panda_gym_amd import _native
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_default_model

    txt, _ = gen_default_model.render()
    assert txt == open(gen_default_model.OUT).read(), "run python tools/gen_default_model.py"
    lib = _native.load()
    params = abi.default_sim_params()
    params.dt *= 2
    cfg = abi.make_config(abi.EnvSpec(), 8, abi.make_model(load_model("panda_custom0")), params)
    h = C.c_void_p()
    assert lib.pgx_create(C.byref(cfg), 0, C.byref(h)) == -3   # PGX_E_UNSUPPORTED
    assert b"compiled for" in lib.pgx_last_error()
    # the scene's table box is part of the block too (round 6): another table, centre or plane top
    for field, k, v in (("table_center", 2, -0.25), ("table_half", 0, 0.6), ("plane_z", None, -0.5)):
        cfg = abi.make_config(abi.EnvSpec(), 8, abi.make_model(load_model("panda_custom0")), abi.default_sim_params())
        if k is None:
            setattr(cfg, field, v)
        else:
            getattr(cfg, field)[k] = v
        assert lib.pgx_create(C.byref(cfg), 0, C.byref(h)) == -3, field
        assert b"compiled for" in lib.pgx_last_error()
    # the substep count is a runtime loop bound, not part of the block
    params = abi.default_sim_params(n_substeps=1)
    cfg = abi.make_config(abi.EnvSpec(), 8, abi.make_model(load_model("panda_custom0")), params)
    rc = lib.pgx_create(C.byref(cfg), 0, C.byref(h))
    assert rc != -3 or b"compiled for" not in lib.pgx_last_error()
    if rc == 0:
        lib.pgx_destroy(h)


def test_constants_match_header():
    hdr = open(os.path.join(ROOT, "include", "pgx.h")).read()

    def define(name):
        return int(re.search(rf"#define {name} (\d+)", hdr).group(1))

    from oracle import oracle as orc

    for name in ("OBJECT_POINTS", "ROBOT_POINTS", "ROBOT_POINTS_ARM", "ROBOT_POINTS_ONE_LANE", "MANIFOLD_POOL",
                 "MANIFOLD_POOL_AO", "MANIFOLD_POINT", "PCG64_WORDS"):
        assert getattr(abi, name) == define("PGX_" + name), name
    assert orc.OBJECT_POINTS == abi.OBJECT_POINTS and orc.ROBOT_MAX >= abi.ROBOT_POINTS
    for name in ("PGX_E_INVALID", "PGX_E_HIP", "PGX_E_UNSUPPORTED", "PGX_E_NOMEM"):
        assert getattr(abi, name) == int(re.search(rf"#define {name} (-\d+)", hdr).group(1)), name
    assert abi.AO_OBSTACLES == define("PGX_AO_OBSTACLES") and abi.MAX_CAPSULES == define("PGX_MAX_CAPSULES")


def test_struct_layout_matches_c(tmp_path):
    """ctypes mirror == C layout of include/pgx.h (sizeof/offsetof via gcc)."""
    src = tmp_path / "lay.c"
    fields = {"pgx_model": ["n_rows", "jpos", "jrot", "mass", "lower", "upper"],
              "pgx_sim_params": ["dt", "ik_max_angle", "n_substeps", "flags"],
              "pgx_config": ["no_auto_reset", "seed", "base_pos", "joint_forces", "model", "params",
                             "terminate_on_success", "collision_reward", "ao_ee_neutral"],
              "pgx_step_out": ["terminal_achieved_goal", "terminal_desired_goal"],
              "pgx_replay_config": ["reward_type", "distance_threshold", "her_ratio", "seed"],
              "pgx_transition": ["next_obs", "done", "timeout"],
              "pgx_replay_batch": ["rows", "env", "goal_slot"], "pgx_state_view": ["episode", "errors", "robot_points"]}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{ROOT}/include/pgx.h"', "int main(){"]
    for s, fs in fields.items():
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for f in fs:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    lines.append("return 0;}")
    src.write_text("\n".join(lines))
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    out = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                          check=True).stdout.split("\n") if l)
    py = {"pgx_model": abi.PgxModel, "pgx_sim_params": abi.PgxSimParams, "pgx_config": abi.PgxConfig,
          "pgx_step_out": abi.PgxStepOut, "pgx_state_view": abi.PgxStateView,
          "pgx_replay_config": abi.PgxReplayConfig, "pgx_transition": abi.PgxTransition,
          "pgx_replay_batch": abi.PgxReplayBatch}
    for s, cls in py.items():
        assert int(out[s]) == C.sizeof(cls), s
        for f in fields[s]:
            assert int(out[f"{s}.{f}"]) == getattr(cls, f).offset, (s, f)
