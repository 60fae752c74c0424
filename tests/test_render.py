"""rgb_array renderer (gym_usv_amd/render.py), the counterpart of SimpleEnvVisualizer.render_frame
(simple_env_visualizer.py:17-113).  pygame is absent, so pixel parity with the reference is
unpinned; these checks fix the canvas, colours, placement and drawing order."""
import numpy as np

from gym_usv_amd.render import render_frame


def _frame():
    readings = np.full(128, 100.0)
    readings[64] = 2.0                                  # the ray straight ahead (psi) hits at 2 m
    obst = np.array([[5.0, 15.0, 0.5]])
    return render_frame((10.0, 10.0, 0.0), (4.0, 4.0), readings, obst, (10.0, 10.0), (110.0, 10.0))


def test_canvas_and_layers():
    img = _frame()
    s = 512 / 20
    assert img.shape == (512, 512, 3) and img.dtype == np.uint8
    assert tuple(img[0, 511]) == (255, 255, 255)                         # background
    assert tuple(img[int(4 * s), int(4 * s)]) == (0, 0, 255)             # target disc
    assert tuple(img[int(15 * s), int(5 * s)]) == (0, 100, 0)            # obstacle (row = y, col = x)
    # the path is drawn last, over the boat: on the path row at x = 10 m
    assert tuple(img[int(10 * s), int(10 * s)]) == (100, 0, 0)
    assert tuple(img[int(10 * s) - 9, int(10 * s)]) == (255, 0, 0)       # boat disc, clear of the front marker
    # a ray pixel beyond the path line width, inside the 2 m ahead ray? ray 64 runs along +x on
    # the path row, so look at a side ray: ray 0 (psi - 120 deg) reaches 100 m, off-canvas
    col = int((10 + 3 * np.cos(-2 * np.pi / 3)) * s)
    row = int((10 + 3 * np.sin(-2 * np.pi / 3)) * s)
    assert tuple(img[row, col]) == (0, 255, 0)


def test_front_marker_follows_heading():
    r = np.full(128, 0.0)
    a = render_frame((10.0, 10.0, np.pi / 2), (0.0, 0.0), r, np.zeros((0, 3)), (0.0, 0.0), (0.0, 0.0))
    s = 512 / 20
    # front disc (olive, 8 px) centred 0.1 m = 2.56 px towards +y, drawn over the boat's disc
    assert tuple(a[int(10 * s + 2.56 + 7), int(10 * s)]) == (100, 100, 0)
