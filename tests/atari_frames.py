"""Atari-like synthetic frame stacks for parity tests (test infrastructure).

Real Breakout frames (gym's 84x84 grayscale pipeline, RL/history.py:29-38 stacks 4 of them)
are mostly large constant regions: a black or grey background, a grey wall, rows of
uniformly coloured bricks, a paddle and a 2x2 ball that move between the 4 history frames.
Constant regions make the 2x2 max-pool windows of every layer tie EXACTLY (MaxPoolGrad must
route to the first maximum, models/pool.py:14-33), and the per-image
max |x| that the scaled-fp16 split derives its exponent from is set by a few bright pixels.
gym/ALE are not installable here, so these frames are drawn, not rendered; the palette is
Breakout's grey levels.
"""
import numpy as np

BRICK_LEVELS = (200, 180, 162, 134, 110, 72)
WALL = 142
BRIGHT = 200


def atari_frames(B, seed, C=4, grey_fraction=0.5):
    """uint8 [B, 84, 84, C]: history channel k is frame t-(C-1)+k of a moving scene."""
    rs = np.random.RandomState(seed)
    out = np.zeros((B, 84, 84, C), np.uint8)
    for n in range(B):
        bg = 87 if rs.uniform() < grey_fraction else 0
        base = np.full((84, 84), bg, np.uint8)
        base[0:6, :] = WALL                              # top wall
        base[:, 0:4] = WALL                              # side walls
        base[:, 80:84] = WALL
        for r, lvl in enumerate(BRICK_LEVELS):           # 6 brick rows of 3 pixels
            y = 14 + 3 * r
            base[y:y + 3, 4:80] = lvl
            for _ in range(rs.randint(0, 6)):            # knocked-out bricks
                x = 4 + 8 * rs.randint(0, 9)
                base[y:y + 3, x:x + 8] = bg
        px, bx, by = rs.randint(8, 64), rs.randint(8, 72), rs.randint(36, 70)
        dpx, dbx, dby = rs.randint(-3, 4), rs.choice([-2, 2]), rs.choice([-3, 3])
        for k in range(C):
            f = base.copy()
            x = int(np.clip(px + k * dpx, 4, 64))
            f[76:78, x:x + 16] = BRIGHT                  # paddle
            yb, xb = by + k * dby, bx + k * dbx
            f[yb:yb + 2, xb:xb + 2] = BRIGHT             # ball
            out[n, :, :, k] = f
    return out
