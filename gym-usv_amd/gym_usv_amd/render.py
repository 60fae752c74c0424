"""rgb_array frames of one env from a state snapshot.

Counterpart of the reference's ``SimpleEnvVisualizer.render_frame``
(gym_usv/envs/simple_env_visualizer.py:17-113, called by ``UsvSimpleEnv.render``,
simple_env.py:117-131) for ``VecVideoRecorder``: a NumPy rasteriser on the host, off the step
path.  Same canvas (512 px for the 20 m field, white), colours, sizes and drawing order: target
(blue, 10 px), the 128 lidar rays (green), the boat (red, 10 px) and its "front" (olive, 8 px,
0.1 m ahead), obstacles (dark green, radius to scale), the path (dark red, 5 px).  Pixel (col,
row) = (x, y) * scale, as pygame's surface transposed to [row, col] by the reference.

Not pinned: pygame, which the reference draws with, is not installed here, so pixel parity with
its anti-aliasing / circle rasterisation is unchecked.  The target after a reset is the path
start (the reference's random reset target is not part of the device state); after a step it is
the closest path point with the lookahead, as in the reference.
"""
from __future__ import annotations

import numpy as np

SENSOR_COUNT = 128
SENSOR_START = -np.pi * 2 / 3                      # usv_asmc_ca_env.py:420
SENSOR_RES = (2 / 3) * (2 * np.pi) / SENSOR_COUNT  # simple_env.py:12-14
BOUND = 20.0                                       # simple_env.py:56


def _disc(img, cx, cy, rad, color):
    h, w, _ = img.shape
    r = max(float(rad), 0.5)
    x0, x1 = int(max(0, np.floor(cx - r))), int(min(w - 1, np.ceil(cx + r)))
    y0, y1 = int(max(0, np.floor(cy - r))), int(min(h - 1, np.ceil(cy + r)))
    if x0 > x1 or y0 > y1:
        return
    yy, xx = np.mgrid[y0:y1 + 1, x0:x1 + 1]
    m = (xx - cx) ** 2 + (yy - cy) ** 2 <= r * r
    img[y0:y1 + 1, x0:x1 + 1][m] = color


def _line(img, p0, p1, color, width=1):
    h, w, _ = img.shape
    n = int(np.ceil(max(abs(p1[0] - p0[0]), abs(p1[1] - p0[1])))) + 1
    n = min(n, 4 * (h + w))
    t = np.linspace(0.0, 1.0, n)
    xs = p0[0] + (p1[0] - p0[0]) * t
    ys = p0[1] + (p1[1] - p0[1]) * t
    half = (width - 1) // 2
    for ox in range(-half, width - half):
        for oy in range(-half, width - half):
            c = np.rint(xs).astype(np.int64) + ox
            r = np.rint(ys).astype(np.int64) + oy
            ok = (c >= 0) & (c < w) & (r >= 0) & (r < h)
            img[r[ok], c[ok]] = color


def render_frame(position, target, readings, obstacles, path_start, path_end, window_size=512):
    """One frame: position (x, y, psi), target (x, y), readings [128] (m), obstacles [n, 3]
    (x, y, r), path start / end (x, y).  Returns uint8 [window_size, window_size, 3]."""
    img = np.full((window_size, window_size, 3), 255, dtype=np.uint8)
    s = window_size / BOUND
    x, y, psi = (float(v) for v in position)
    _disc(img, target[0] * s, target[1] * s, 10, (0, 0, 255))
    ang = SENSOR_START + np.arange(SENSOR_COUNT) * SENSOR_RES + psi       # sensor_data[:, 0]
    for a, d in zip(ang, readings):
        _line(img, (x * s, y * s), ((d * np.cos(a) + x) * s, (d * np.sin(a) + y) * s), (0, 255, 0))
    _disc(img, x * s, y * s, 10, (255, 0, 0))
    _disc(img, (x + 0.1 * np.cos(psi)) * s, (y + 0.1 * np.sin(psi)) * s, 8, (100, 100, 0))
    for ox, oy, r in obstacles:
        _disc(img, ox * s, oy * s, r * s, (0, 100, 0))
    _line(img, (path_start[0] * s, path_start[1] * s), (path_end[0] * s, path_end[1] * s), (100, 0, 0), width=5)
    return img


def frame_from_state(fields, i, obs_row, window_size=512):
    """Frame of env i from get_field arrays (x, y, psi, path_*, progress, n_obs, obs_x/y/r) and
    its current obs row (sensors = obs[15:] * 100)."""
    p0 = np.array([fields["path_x0"][i], fields["path_y0"][i]])
    p1 = np.array([fields["path_x1"][i], fields["path_y1"][i]])
    target = p0 + float(fields["progress"][i]) * (p1 - p0)      # closest point (simple_env.py:139-148)
    n = int(fields["n_obs"][i])
    obst = np.stack([fields["obs_x"][i, :n], fields["obs_y"][i, :n], fields["obs_r"][i, :n]], axis=1)
    readings = np.asarray(obs_row[15:15 + SENSOR_COUNT], dtype=np.float64) * 100.0
    pos = (fields["x"][i], fields["y"][i], fields["psi"][i])
    return render_frame(pos, target, readings, obst, p0, p1, window_size)
