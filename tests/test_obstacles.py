"""Obstacle messages -> solver inputs (obstacles.py): the
ObstacleGMM / ObstacleArray handling, the time shift of received robot plans,
the merge into the obstacle list, padding / closest-first selection and the
ellipsoid parameter arrays.  Known answers are derived by hand from the
reference lines each function cites (the reference has no tests for them)."""
import math

import numpy as np
import pytest

from oscar_mpc_planner_mr_modification_amd import obstacles as ob


def _line_plan(x0, y0, vx, vy, N, dt, t0=0.0):
    pos = [(x0 + vx * (t0 + k * dt), y0 + vy * (t0 + k * dt)) for k in range(N)]
    ang = [math.atan2(vy, vx)] * N
    return pos, ang


def test_angles_and_quaternions():
    for psi in (-3.0, -1.0, 0.0, 0.7, 3.1):
        assert abs(ob.quaternion_to_angle(ob.angle_to_quaternion(psi)) - psi) < 1e-12
    assert abs(ob.wrap_angle(3 * math.pi) - math.pi) < 1e-12
    assert abs(ob.wrap_angle(-7.0) - (-7.0 + 2 * math.pi)) < 1e-12
    # shortest arc across +-pi
    a = ob.interpolate_angle(3.0, -3.0, 0.5)
    assert abs(abs(a) - math.pi) < 1e-12
    assert abs(ob.interpolate_angle(0.2, 0.6, 0.25) - 0.3) < 1e-12
    assert abs(ob.exponential_quantile(0.5, 0.95) - (-2.0 * math.log(0.05))) < 1e-12


def test_trajectory_message_round_trip_and_id_check():
    N, dt = 30, 0.2
    pos, ang = _line_plan(1.0, 2.0, 0.5, -0.25, N, dt)
    msg = ob.direct_trajectory_msg(2, (1.0, 2.0, ang[0]), pos, ang, dt, stamp=10.0)
    robot = ob.DynamicObstacle(2, (100.0, 100.0), 0.0, 0.325)
    assert ob.apply_trajectory_msg(robot, msg, now=10.0)
    assert robot.prediction_type == ob.DETERMINISTIC and len(robot.mode) == N
    np.testing.assert_allclose(robot.mode.positions, pos, rtol=0, atol=1e-15)
    np.testing.assert_allclose(robot.mode.angles, ang, rtol=0, atol=1e-12)
    assert robot.mode.major == [-1.0] * N
    other = ob.DynamicObstacle(1, (100.0, 100.0), 0.0, 0.325)
    assert not ob.apply_trajectory_msg(other, msg, now=10.0)          # id mismatch: ignored
    assert not ob.apply_trajectory_msg(robot, dict(msg, gaussians=[]), now=10.0)


@pytest.mark.parametrize("elapsed", [0.3, 0.2, 0.47, 1.0])
def test_time_shift_of_a_constant_velocity_plan_is_exact(elapsed):
    """k = floor(el/dt) steps dropped, k+1 extrapolated, fractional interpolation:
    for a straight constant-velocity plan the result is the plan evaluated at t + el."""
    N, dt = 30, 0.2
    pos, ang = _line_plan(0.0, 0.0, 1.0, 0.5, N, dt)
    o = ob.DynamicObstacle(0, pos[0], ang[0], 0.3)
    for p, a in zip(pos, ang):
        o.mode.append(p, a, -1, -1)
    o.last_update_time = 5.0
    assert ob.interpolate_by_elapsed_time(o, 5.0 + elapsed, N, dt, 20.0)
    want, _ = _line_plan(0.0, 0.0, 1.0, 0.5, N, dt, t0=elapsed)
    np.testing.assert_allclose(o.mode.positions, want, rtol=0, atol=1e-12)
    assert o.position == o.mode.positions[0] and o.last_update_time == 5.0 + elapsed


def test_time_shift_skips_fresh_stale_and_wrong_length():
    N, dt = 30, 0.2
    pos, ang = _line_plan(0.0, 0.0, 1.0, 0.0, N, dt)

    def make(n=N):
        o = ob.DynamicObstacle(0, pos[0], 0.0, 0.3, last_update_time=1.0)
        for p, a in list(zip(pos, ang))[:n]:
            o.mode.append(p, a, -1, -1)
        return o
    for now in (1.0 + 0.04, 1.0 + N * dt + 0.1):       # fresher than one control period / beyond the horizon
        o = make()
        assert not ob.interpolate_by_elapsed_time(o, now, N, dt, 20.0)
        assert o.mode.positions == pos
    o = make(N - 1)
    assert not ob.interpolate_by_elapsed_time(o, 1.5, N, dt, 20.0)


def test_time_shift_clamps_the_extrapolation_speed():
    N, dt = 10, 0.2
    pos, ang = _line_plan(0.0, 0.0, 5.0, 0.0, N, dt)     # 5 m/s > robot_max_velocity 2
    o = ob.DynamicObstacle(0, pos[0], 0.0, 0.3, last_update_time=0.0)
    for p, a in zip(pos, ang):
        o.mode.append(p, a, -1, -1)
    assert ob.interpolate_by_elapsed_time(o, 0.4, N, dt, 20.0, v_max=2.0)
    xs = [p[0] for p in o.mode.positions]
    np.testing.assert_allclose(xs[:N - 2], [5.0 * dt * (k + 2) for k in range(N - 2)], atol=1e-12)
    last = 5.0 * dt * (N - 1)
    np.testing.assert_allclose(xs[N - 2:], [last + 2.0 * dt, last + 2.0 * 2 * dt], atol=1e-12)


def test_merge_pad_and_keep_closest():
    N, dt = 20, 0.2
    state = (0.0, 0.0, 0.0, 1.0)
    near = ob.DynamicObstacle(7, (2.0, 0.0), 0.0, 0.325)
    near.prediction_type, near.mode = ob.constant_velocity_prediction((2.0, 0.0), (0.0, 0.0), dt, N)
    robot = ob.DynamicObstacle(1, (5.0, 0.0), 0.0, 0.325)
    robot.prediction_type, robot.mode = ob.constant_velocity_prediction((5.0, 1.0), (0.0, 0.0), dt, N)
    merged = ob.update_robot_obstacles([near], {"/jackal2": robot, "/jackal3": ob.DynamicObstacle(2, (0, 0), 0, 1)},
                                       validated={"/jackal2"})
    assert [o.index for o in merged] == [7, 1]
    padded = ob.ensure_obstacle_size(merged, state, 4, N, dt)
    assert len(padded) == 4 and padded[2].index == -1
    assert padded[3].position == (100.0, 100.0) and padded[3].radius == 0.0
    far = [ob.DynamicObstacle(10 + i, (40.0 + i, 0.0), 0.0, 0.3) for i in range(3)]
    for f in far:
        f.prediction_type, f.mode = ob.constant_velocity_prediction(f.position, (0.0, 0.0), dt, N)
    kept = ob.ensure_obstacle_size(far + merged, state, 2, N, dt)
    assert [o.position for o in kept] == [(2.0, 0.0), (5.0, 0.0)]
    assert [o.index for o in kept] == [0, 1]                  # sequential ids after the cut


def test_obstacle_array_typing_and_ellipsoid_arrays():
    N, dt = 20, 0.2
    pos, ang = _line_plan(3.0, 1.0, 0.3, 0.0, N, dt)
    det = ob.obstacle_gmm_msg(0, 3.0, 1.0, 0.0, pos, ang, major=[0.0] * N, minor=[0.0] * N)
    gau = ob.obstacle_gmm_msg(1, 3.0, 1.0, 0.0, pos, ang, major=[0.2] * N, minor=[0.1] * N)
    none = dict(ob.obstacle_gmm_msg(2, 9.0, 9.0, 0.0, pos, ang), probabilities=[])
    obs = ob.obstacles_from_array({"obstacles": [det, gau, none]}, 0.325, probabilistic=True)
    assert [o.prediction_type for o in obs[:2]] == [ob.DETERMINISTIC, ob.GAUSSIAN]
    assert len(obs[2].mode) == 0
    assert ob.obstacles_from_array({"obstacles": [gau]}, 0.325)[0].prediction_type == ob.DETERMINISTIC
    arr, meta = ob.scene_obstacle_arrays(obs[:2], N)
    np.testing.assert_allclose(arr[0, :, 0:2], pos, atol=1e-15)
    assert (arr[0, :, 3:5] == 0).all() and meta[0].tolist() == [0.325, 1.0]
    assert np.allclose(arr[1, :, 3], 0.2) and abs(meta[1, 1] - ob.exponential_quantile(0.5, 0.95)) < 1e-15
    with pytest.raises(ValueError):
        ob.obstacles_from_array({"obstacles": [dict(gau, probabilities=[0.5, 0.5])]}, 0.3)


def test_recording_replay_through_the_tracker(tmp_path):
    """Three robots: the ego (jackal1) replays plans of jackal2 / jackal3 received at
    different times; the prepared list is the shifted robot plans + array obstacles + dummies."""
    N, dt = 30, 0.2
    steps = []
    for t_i, t in enumerate((0.0, 0.05, 0.1)):
        p2, a2 = _line_plan(4.0, 0.0, -0.5, 0.0, N, dt, t0=0.0)
        p3, a3 = _line_plan(0.0, 4.0, 0.0, -0.5, N, dt, t0=0.0)
        msgs = {}
        if t_i == 0:
            msgs["/jackal2"] = ob.direct_trajectory_msg(1, (4.0, 0.0, a2[0]), p2, a2, dt, stamp=t)
        if t_i == 1:
            msgs["/jackal3"] = ob.direct_trajectory_msg(2, (0.0, 4.0, a3[0]), p3, a3, dt, stamp=t)
        arr = {"obstacles": [ob.obstacle_gmm_msg(5, 8.0, 8.0, 0.0, *_line_plan(8.0, 8.0, 0.0, 0.0, N, dt))]}
        steps.append({"t": t, "state": [0.0, 0.0, 0.0, 1.0, 0.0], "obstacle_array": arr, "robot_msgs": msgs})
    path = tmp_path / "rec.jsonl"
    ob.write_recording(str(path), steps)
    rec = ob.read_recording(str(path))
    assert rec == steps
    tr = ob.RobotObstacleTracker(["/jackal1", "/jackal2", "/jackal3"], "/jackal1", 0.325, N, dt, max_obstacles=6)
    for s in rec:
        for ns, m in s["robot_msgs"].items():
            tr.on_trajectory(ns, m, s["t"])
        lst = tr.prepare(ob.obstacles_from_array(s["obstacle_array"], 0.325), s["state"], s["t"])
    assert [o.index for o in lst] == [5, 1, 2, -1, -1, -1]
    # jackal2's plan was received at t = 0 and is shifted by 0.1 s at t = 0.1
    np.testing.assert_allclose(lst[1].mode.positions[0], (4.0 - 0.5 * 0.1, 0.0), atol=1e-12)
    # jackal3's plan is 0.05 s old (not fresher than one 20 Hz period): k = 0, alpha = 0.25
    np.testing.assert_allclose(lst[2].mode.positions[0], (0.0, 4.0 - 0.5 * 0.05), atol=1e-12)
    obst, meta = ob.scene_obstacle_arrays(lst, N)
    assert obst.shape == (6, N, 5) and (meta[3:] == [0.0, 1.0]).all()


@pytest.mark.gpu
def test_replayed_multi_robot_scene_through_the_gpu_step(oracle_mod):
    """C4 scenes whose obstacle lists come from replayed robot plans (tracker) plus
    array obstacles: GPU producer bit-exact against the host producer on the
    ellipsoid rows, GPU solve against the oracle."""
    import torch
    from oscar_mpc_planner_mr_modification_amd import native
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    from oscar_mpc_planner_mr_modification_amd.producers import prepare_host
    from oscar_mpc_planner_mr_modification_amd.synthetic import (DECELERATION, ROBOT_RADIUS, SETTINGS_WEIGHTS,
                                                                 make_scenes)
    lay = config_layout("C4")
    N, dt = lay.N, lay.dt
    S, G = 3, 8
    sc = make_scenes(lay, S, G, n_obs=lay.n_ell, seed=4711)
    for s in range(S):
        x0 = sc.state[s]
        tr = ob.RobotObstacleTracker(["/jackal1", "/jackal2", "/jackal3", "/jackal4"], "/jackal1", 0.325, N, dt,
                                     max_obstacles=lay.n_ell)
        for r, ns in enumerate(("/jackal2", "/jackal3", "/jackal4")):
            start = (x0[0] + 3.0 + r, x0[1] - 1.5 + 1.5 * r)
            pos, ang = _line_plan(start[0], start[1], -0.4, 0.1 * (r - 1), N, dt)
            tr.on_trajectory(ns, ob.direct_trajectory_msg(r + 1, (*start, ang[0]), pos, ang, dt, stamp=0.0), 0.0)
        arr = ob.obstacles_from_array({"obstacles": [
            ob.obstacle_gmm_msg(10 + j, x0[0] + 5 + j, x0[1] + 2 - j, 0.0,
                                *_line_plan(x0[0] + 5 + j, x0[1] + 2 - j, -0.3, 0.0, N, dt))
            for j in range(5)]}, 0.325)
        lst = tr.prepare(arr, x0, now=0.13)
        sc.obst[s], sc.obst_meta[s] = ob.scene_obstacle_arrays(lst, N)
    host = prepare_host(lay, sc, ROBOT_RADIUS, SETTINGS_WEIGHTS["consistency"], DECELERATION)
    dev = torch.device("cuda:0")
    pr = native.problem_from_layout(lay)
    out = native.prepare_device(pr, native.scenes_to_device(sc, dev), ROBOT_RADIUS, SETTINGS_WEIGHTS["consistency"],
                                DECELERATION)
    got = native.solve_batch_device(pr, out["params"], out["warm"], out["xinit"])
    torch.cuda.synchronize()
    prm = out["params"].cpu().numpy()
    np.testing.assert_array_equal(prm, host.params)
    ref = oracle_mod.Oracle(lay).solve_batch(prm, out["warm"].cpu().numpy(), out["xinit"].cpu().numpy())
    ex = got["exit"].cpu().numpy()
    assert np.array_equal(ex, ref["status"])
    ok = ex == 1
    assert ok.any()
    assert np.abs(got["xtraj"].cpu().numpy()[ok] - ref["xtraj"][ok]).max() <= 1e-4
