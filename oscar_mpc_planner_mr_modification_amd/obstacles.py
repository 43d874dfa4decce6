"""Obstacle messages and their preparation for the solve.

The C4 workload (jackal multi-robot) plans around other robots whose plans
arrive as `mpc_planner_msgs/ObstacleGMM` messages and around
non-communicating obstacles that arrive in an `ObstacleArray`. This module
restates, host side, what the reference does with those messages before the
per-guess solves, so that recorded (or synthetic) message streams can be
replayed through the batched GPU control step:

  message types         mpc_planner_msgs/msg/{ObstacleGMM,Gaussian,ObstacleArray}.msg,
                        kept as dicts with the ROS field names (JSON-lines recordings)
  ObstacleArray -> obstacles       JackalPlanner::obstacleCallback (ros1_jackalsimulator.cpp:299-353)
  ObstacleGMM  -> robot obstacle   JulesJackalPlanner::trajectoryCallback (jules_ros1_jackalplanner.cpp:521-640)
  plan         -> ObstacleGMM      JulesJackalPlanner::publishDirectTrajectory (:1265-1320)
  time shift of a received plan    interpolateTrajectoryPredictionsByTime (:840-1064),
                                   MultiRobot::{wrapAngle, interpolateAngle} (multi_robot_utility_functions.cpp:127-157)
  merge into the obstacle list     MultiRobot::updateRobotObstaclesFromTrajectories (data_preparation.cpp:202-237)
  pad / keep the closest           ensureObstacleSize, getDummyObstacle, getConstantVelocityPrediction,
                                   propagatePredictionUncertainty (data_preparation.cpp:55-200)
  obstacles -> solver arrays       EllipsoidConstraints::setParameters (ellipsoid_constraints.cpp:34-86):
                                   the `obst` / `obst_meta` buffers of mpcg_scene_io (include/mpcg.h)

`RosTools::quaternionToAngle` / `angleToQuaternion` and `ExponentialQuantile`
live in the external ros_tools package and are restated as the standard yaw
extraction and the exponential-distribution quantile (parity unpinned there).
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass, field

import numpy as np

# ---------------------------------------------------------------- ros_tools


def quaternion_to_angle(q: dict) -> float:
    """Yaw of a quaternion {x, y, z, w} (RosTools::quaternionToAngle)."""
    x, y, z, w = (float(q.get(k, 0.0)) for k in ("x", "y", "z", "w"))
    return math.atan2(2.0 * (w * z + x * y), 1.0 - 2.0 * (y * y + z * z))


def angle_to_quaternion(psi: float) -> dict:
    """Planar yaw as a quaternion (RosTools::angleToQuaternion)."""
    return {"x": 0.0, "y": 0.0, "z": math.sin(0.5 * psi), "w": math.cos(0.5 * psi)}


def exponential_quantile(lam: float, p: float) -> float:
    """Quantile p of an exponential distribution with rate lam (RosTools::ExponentialQuantile)."""
    return -math.log(1.0 - p) / lam


# ------------------------------------------------- multi_robot_utility_functions.cpp


def wrap_angle(angle: float) -> float:
    """MultiRobot::wrapAngle (:143-150): loop into [-pi, pi]."""
    while angle > math.pi:
        angle -= 2.0 * math.pi
    while angle < -math.pi:
        angle += 2.0 * math.pi
    return angle


def interpolate_angle(psi_k: float, psi_kl: float, alpha: float) -> float:
    """MultiRobot::interpolateAngle (:127-140): along the shortest arc."""
    return wrap_angle(psi_k + wrap_angle(psi_kl - psi_k) * alpha)


# ------------------------------------------------------------------ data types

DETERMINISTIC, GAUSSIAN = 0, 1   # PredictionType (data_types.h:35-41)


@dataclass
class Mode:
    """One prediction mode: per step position, angle, major/minor radius (data_types.h:43-60)."""
    positions: list = field(default_factory=list)
    angles: list = field(default_factory=list)
    major: list = field(default_factory=list)
    minor: list = field(default_factory=list)

    def __len__(self):
        return len(self.positions)

    def append(self, pos, angle, major, minor):
        self.positions.append((float(pos[0]), float(pos[1])))
        self.angles.append(float(angle))
        self.major.append(float(major))
        self.minor.append(float(minor))


@dataclass
class DynamicObstacle:
    """data_types.h:85-109 (ros::Time replaced by seconds)."""
    index: int
    position: tuple
    angle: float
    radius: float
    prediction_type: int = DETERMINISTIC
    mode: Mode = field(default_factory=Mode)
    last_update_time: float = 0.0
    needs_interpolation: bool = False


def constant_velocity_prediction(position, velocity, dt: float, steps: int, probabilistic: bool = False):
    """getConstantVelocityPrediction (data_preparation.cpp:62-81)."""
    noise = 0.3 if probabilistic else 0.0
    m = Mode()
    for i in range(steps):
        m.append((position[0] + velocity[0] * dt * i, position[1] + velocity[1] * dt * i), 0.0, noise, noise)
    kind = GAUSSIAN if probabilistic else DETERMINISTIC
    if probabilistic:
        propagate_uncertainty(kind, m, dt, steps)
    return kind, m


def propagate_uncertainty(kind: int, mode: Mode, dt: float, N: int):
    """propagatePredictionUncertainty (data_preparation.cpp:174-191): integrate the per-step
    standard deviations over the horizon."""
    if kind != GAUSSIAN:
        return
    major = minor = 0.0
    for k in range(N):
        major = math.sqrt(major ** 2 + (mode.major[k] * dt) ** 2)
        minor = math.sqrt(minor ** 2 + (mode.minor[k] * dt) ** 2)
        mode.major[k] = major
        mode.minor[k] = minor


def dummy_obstacle(state, N: int, dt: float, probabilistic: bool = False) -> DynamicObstacle:
    """getDummyObstacle + zero-velocity prediction (data_preparation.cpp:55-60, 155-170)."""
    o = DynamicObstacle(-1, (state[0] + 100.0, state[1] + 100.0), 0.0, 0.0)
    o.prediction_type, o.mode = constant_velocity_prediction(o.position, (0.0, 0.0), dt, N, probabilistic)
    return o


def ensure_obstacle_size(obstacles: list, state, max_obstacles: int, N: int, dt: float,
                         probabilistic: bool = False) -> list:
    """ensureObstacleSize (data_preparation.cpp:97-172): keep the `max_obstacles`
    closest (a horizon-weighted distance to a constant-velocity roll-out of the
    ego state, stable sort) and renumber them, or pad with dummies.
    state = (x, y, psi, v, ...)."""
    obstacles = list(obstacles)
    if len(obstacles) > max_obstacles:
        dirx, diry = math.cos(state[2]), math.sin(state[2])
        dist = []
        for o in obstacles:
            best = 1e5
            for k in range(N):
                px, py = o.mode.positions[k]
                ex, ey = state[0] + state[3] * k * dirx, state[1] + state[3] * k * diry
                d = (k + 1) * 0.6 * math.hypot(px - ex, py - ey)
                best = min(best, d)
            dist.append(best)
        order = sorted(range(len(obstacles)), key=lambda i: dist[i])
        obstacles = [obstacles[i] for i in order[:max_obstacles]]
        for i, o in enumerate(obstacles):
            o.index = i
    while len(obstacles) < max_obstacles:
        obstacles.append(dummy_obstacle(state, N, dt, probabilistic))
    return obstacles


# ------------------------------------------------------------------ messages


def _pose(x, y, psi, z=0.0):
    return {"position": {"x": float(x), "y": float(y), "z": float(z)}, "orientation": angle_to_quaternion(psi)}


def obstacle_gmm_msg(index: int, x: float, y: float, psi: float, positions, angles, major=None, minor=None,
                     stamp: float = 0.0, dt: float = 0.2) -> dict:
    """An ObstacleGMM with one Gaussian (mean path + semi-axes), as a dict with the ROS field names."""
    n = len(positions)
    major = [-1.0] * n if major is None else list(major)
    minor = [-1.0] * n if minor is None else list(minor)
    poses = [{"header": {"stamp": stamp + k * dt}, "pose": _pose(p[0], p[1], a, k * dt)}
             for k, (p, a) in enumerate(zip(positions, angles))]
    return {"id": int(index), "pose": _pose(x, y, psi),
            "gaussians": [{"mean": {"header": {"stamp": stamp}, "poses": poses},
                           "major_semiaxis": major, "minor_semiaxis": minor}],
            "probabilities": [1.0]}


def direct_trajectory_msg(ego_id: int, state, positions, orientations, dt: float, stamp: float) -> dict:
    """JulesJackalPlanner::publishDirectTrajectory (jules_ros1_jackalplanner.cpp:1265-1320):
    the ego plan as an ObstacleGMM, dummy semi-axes -1, pose z = k dt."""
    return obstacle_gmm_msg(ego_id, state[0], state[1], state[2], positions, orientations, stamp=stamp, dt=dt)


def obstacles_from_array(msg: dict, obstacle_radius: float, probabilistic: bool = False) -> list:
    """JackalPlanner::obstacleCallback (ros1_jackalsimulator.cpp:299-345), before
    ensureObstacleSize: one obstacle per ObstacleGMM, its single Gaussian mode as the
    prediction (DETERMINISTIC when the last major semi-axis is 0 or probabilistic is off)."""
    out = []
    for ob in msg["obstacles"]:
        p = ob["pose"]["position"]
        o = DynamicObstacle(int(ob["id"]), (float(p["x"]), float(p["y"])), quaternion_to_angle(ob["pose"]["orientation"]),
                            obstacle_radius)
        out.append(o)
        probs = ob.get("probabilities", [])
        if len(probs) == 0:
            continue   # no prediction
        if len(probs) != 1:
            raise ValueError("Multiple modes not yet supported")   # ROSTOOLS_ASSERT in the reference
        g = ob["gaussians"][0]
        for k, ps in enumerate(g["mean"]["poses"]):
            pp = ps["pose"]
            o.mode.append((pp["position"]["x"], pp["position"]["y"]), quaternion_to_angle(pp["orientation"]),
                          g["major_semiaxis"][k], g["minor_semiaxis"][k])
        o.prediction_type = DETERMINISTIC if (g["major_semiaxis"][-1] == 0.0 or not probabilistic) else GAUSSIAN
    return out


def apply_trajectory_msg(obs: DynamicObstacle, msg: dict, now: float) -> bool:
    """JulesJackalPlanner::trajectoryCallback (jules_ros1_jackalplanner.cpp:521-640) for a
    robot obstacle in an active planner state: pose update and the message's first Gaussian
    mean as a DETERMINISTIC mode (semi-axes -1). Returns False when the message is ignored
    (no Gaussians or an id mismatch)."""
    if not msg.get("gaussians") or obs.index != int(msg["id"]):
        return False
    p = msg["pose"]["position"]
    obs.position = (float(p["x"]), float(p["y"]))
    obs.angle = quaternion_to_angle(msg["pose"]["orientation"])
    m = Mode()
    for ps in msg["gaussians"][0]["mean"]["poses"]:
        pp = ps["pose"]
        m.append((pp["position"]["x"], pp["position"]["y"]), quaternion_to_angle(pp["orientation"]), -1.0, -1.0)
    obs.prediction_type = DETERMINISTIC
    obs.mode = m
    obs.last_update_time = now
    obs.needs_interpolation = False
    return True


def interpolate_by_elapsed_time(obs: DynamicObstacle, now: float, N: int, dt: float, control_frequency: float,
                                v_max: float = 2.0, w_max: float = 2.0) -> bool:
    """interpolateTrajectoryPredictionsByTime (jules_ros1_jackalplanner.cpp:840-1064) for one
    robot obstacle: shift the received plan by the time since it was received (whole steps
    dropped, k + 1 constant-velocity points extrapolated from the last two, all points
    interpolated by the fractional remainder). Returns True when the plan was shifted."""
    mode = obs.mode
    n = len(mode)
    if n != N:
        return False
    el = now - obs.last_update_time
    if el < 1.0 / control_frequency:
        obs.needs_interpolation = False
        return False
    k = int(math.floor(el / dt))
    tau = el - k * dt
    alpha = tau / dt
    if k >= N:
        obs.needs_interpolation = False     # critically stale: left as is
        return False
    if k == 0 and alpha < 0.01:
        obs.needs_interpolation = False
        return False
    pos = [tuple(p) for p in mode.positions]
    ang = list(mode.angles)
    ext_p, ext_a = [], []
    if n >= 2:
        (lx, ly), (sx, sy) = pos[-1], pos[-2]
        vx, vy = (lx - sx) / dt, (ly - sy) / dt
        psi_dot = wrap_angle(ang[-1] - ang[-2]) / dt
        vm = math.hypot(vx, vy)
        if vm > v_max:
            vx, vy = vx / vm * v_max, vy / vm * v_max
        if abs(psi_dot) > w_max:
            psi_dot = min(max(psi_dot, -w_max), w_max)
        for i in range(1, k + 2):
            te = i * dt
            ext_p.append((lx + vx * te, ly + vy * te))
            ext_a.append(wrap_angle(ang[-1] + psi_dot * te))
    pos = pos[k:] + ext_p
    ang = ang[k:] + ext_a
    if alpha > 0.001:
        ip, ia = [], []
        for i in range(len(pos) - 1):
            (cx, cy), (nx_, ny) = pos[i], pos[i + 1]
            ip.append(((1 - alpha) * cx + alpha * nx_, (1 - alpha) * cy + alpha * ny))
            ia.append(interpolate_angle(ang[i], ang[i + 1], alpha))
        pos, ang = ip, ia
    elif len(pos) > N:
        pos, ang = pos[:-1], ang[:-1]
    while len(pos) < N:
        pos.append(pos[-1])
        ang.append(ang[-1])
    pos, ang = pos[:N], ang[:N]
    m = Mode()
    for p, a in zip(pos, ang):
        m.append(p, a, -1.0, -1.0)
    obs.mode = m
    obs.position = pos[0]
    obs.angle = ang[0]
    obs.needs_interpolation = True
    obs.last_update_time = now
    return True


def update_robot_obstacles(dynamic: list, robots: dict, validated: set) -> list:
    """MultiRobot::updateRobotObstaclesFromTrajectories (data_preparation.cpp:202-237):
    replace the obstacle with the robot's index, or append it; robots that have not sent a
    valid plan yet are skipped.  `robots`: namespace -> DynamicObstacle (iterated in key
    order, like the std::map of the reference)."""
    out = list(dynamic)
    for ns in sorted(robots):
        if ns not in validated:
            continue
        ro = robots[ns]
        for i, o in enumerate(out):
            if o.index == ro.index:
                out[i] = ro
                break
        else:
            out.append(ro)
    return out


def scene_obstacle_arrays(obstacles: list, N: int, risk: float = 0.05):
    """EllipsoidConstraints::setParameters (ellipsoid_constraints.cpp:56-86) as the
    mpcg_scene_io buffers: obst [n][N][5] = mode-0 step k (x, y, angle, major, minor) for
    solver stage k + 1, obst_meta [n][2] = (radius, chi). DETERMINISTIC: major = minor = 0,
    chi = 1; GAUSSIAN: the mode's semi-axes, chi = ExponentialQuantile(0.5, 1 - risk)."""
    n = len(obstacles)
    obst = np.zeros((n, N, 5))
    meta = np.zeros((n, 2))
    chi_g = exponential_quantile(0.5, 1.0 - risk)
    for j, o in enumerate(obstacles):
        det = o.prediction_type == DETERMINISTIC
        for k in range(N):
            kk = min(k, len(o.mode) - 1)
            px, py = o.mode.positions[kk]
            obst[j, k] = (px, py, o.mode.angles[kk], 0.0 if det else o.mode.major[kk],
                          0.0 if det else o.mode.minor[kk])
        meta[j] = (o.radius, 1.0 if det else chi_g)
    return obst, meta


# ------------------------------------------------------------------ recordings


def write_recording(path: str, steps: list):
    """JSON lines, one control step per line: {"t", "state", "obstacle_array", "robot_msgs"}."""
    with open(path, "w") as fh:
        for s in steps:
            fh.write(json.dumps(s) + "\n")


def read_recording(path: str) -> list:
    with open(path) as fh:
        return [json.loads(line) for line in fh if line.strip()]


class RobotObstacleTracker:
    """The multi-robot obstacle state of one planner across control steps
    (jules_ros1_jackalplanner.cpp:100-160 initialisation, :521-640 callbacks,
    :800-850 prepareObstacleData): replay a recording step by step."""

    def __init__(self, robot_namespaces, ego_ns: str, radius: float, N: int, dt: float, max_obstacles: int,
                 control_frequency: float = 20.0, probabilistic: bool = False):
        self.N, self.dt, self.max_obstacles = N, dt, max_obstacles
        self.control_frequency = control_frequency
        self.probabilistic = probabilistic
        self.robots = {}
        self.validated = set()
        for ns in robot_namespaces:
            if ns == ego_ns:
                continue
            idx = int(ns.lstrip("/")[6:]) - 1   # extractRobotIdFromNamespace: jackalX -> X - 1
            self.robots[ns] = DynamicObstacle(idx, (100.0, 100.0), 0.0, radius)

    def on_trajectory(self, ns: str, msg: dict, now: float):
        ro = self.robots.get(ns)
        if ro is not None and apply_trajectory_msg(ro, msg, now):
            self.validated.add(ns)

    def prepare(self, obstacles: list, state, now: float) -> list:
        """prepareObstacleData: shift every robot plan to `now`, merge, pad / keep the closest."""
        for ns in sorted(self.robots):
            interpolate_by_elapsed_time(self.robots[ns], now, self.N, self.dt, self.control_frequency)
        merged = update_robot_obstacles(obstacles, self.robots, self.validated)
        return ensure_obstacle_size(merged, state, self.max_obstacles, self.N, self.dt, self.probabilistic)
