"""The spatial pass's XCD tile order (kernels.hip `xcd_tile` / `xcd_grid`), restated: for the image sizes of the
BASELINE configs and the chunk shapes the knobs allow (spatial.xcd_rows, spatial.xcd_cols), the launch's blocks
visit every tile exactly once, each XCD (block % 8) works on whole chunks, and no block maps outside the image.
CPU only; the GPU parity tests (`test_spatial_pass_bit_exact[ntl_2d*]`) run the device code itself."""
import pytest


def xcd_tile(ntx, T, rows, cols, b):
    x, j = b % 8, b // 8
    if rows == 0:
        q, rem = T // 8, T % 8
        return x * q + min(x, rem) + j, j < q + (1 if x < rem else 0)
    if cols == 0 or cols >= ntx:
        chunk = rows * ntx
        i = j // chunk
        tile = ((x + 8 * i) * rows) * ntx + (j - i * chunk)
        return tile, tile < T
    cw = cols
    ncx = (ntx + cw - 1) // cw
    chunk = rows * cw
    i, k = j // chunk, j % chunk
    c = x + 8 * i
    cr, tr = c // ncx, k // cw
    col = (c - cr * ncx) * cw + (k - tr * cw)
    tile = (cr * rows + tr) * ntx + col
    return tile, col < ntx and tile < T


def xcd_grid(ntx, nty, rows, cols):
    if rows == 0:
        return ntx * nty
    cw = ntx if (cols == 0 or cols >= ntx) else cols
    chunks = ((nty + rows - 1) // rows) * ((ntx + cw - 1) // cw)
    return 8 * ((chunks + 7) // 8) * rows * cw


SIZES = [(1920, 1080, 8), (3840, 2160, 16), (7680, 4320, 8), (96, 64, 8), (960, 1100, 8), (1940, 1100, 8)]
SHAPES = [(0, 0), (1, 0), (2, 0), (4, 0), (4, 30), (8, 30), (2, 2), (4, 15), (8, 20), (16, 15), (3, 7), (1, 1)]


@pytest.mark.parametrize("W,H,th", SIZES)
@pytest.mark.parametrize("rows,cols", SHAPES)
def test_every_tile_once(W, H, th, rows, cols):
    ntx, nty = (W + 31) // 32, (H + th - 1) // th
    T = ntx * nty
    grid = xcd_grid(ntx, nty, rows, cols)
    seen = [0] * T
    owner = {}
    for b in range(grid):
        tile, ok = xcd_tile(ntx, T, rows, cols, b)
        if not ok:
            continue
        assert 0 <= tile < T
        seen[tile] += 1
        if rows and cols and cols < ntx:
            # a chunk (rows x cols tiles) belongs to one XCD
            chunk = (tile // ntx // rows, tile % ntx // cols)
            assert owner.setdefault(chunk, b % 8) == b % 8
    assert seen == [1] * T
