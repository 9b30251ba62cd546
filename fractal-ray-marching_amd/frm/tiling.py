"""Row-band tiling of a frame across ranks: band b (band_rows rows)
goes to rank b % ranks; each rank renders its bands back to back into one buffer of
equal size (padded), the buffers are gathered rank-major on rank 0 and unshuffled.
Pure-Python geometry + a numpy reassembly used by the CPU (gloo) tests; libfrm's
frm_render_bands / frm_unshuffle_bands implement the same layout on the GPU."""
import numpy as np


def num_bands(height, band_rows):
    return (height + band_rows - 1) // band_rows


def bands_of_rank(height, band_rows, rank, ranks):
    return list(range(rank, num_bands(height, band_rows), ranks))


def rank_rows(height, band_rows, rank, ranks):
    """Rows in rank's buffer (whole bands, the last band of the frame padded)."""
    return len(bands_of_rank(height, band_rows, rank, ranks)) * band_rows


def rank_buffer_rows(height, band_rows, ranks):
    """Equal per-rank buffer size for the gather (rank 0 has the most bands)."""
    return rank_rows(height, band_rows, 0, ranks)


def choose_band_rows(height, ranks, target=16):
    """Smallest band height >= target that divides height into a multiple of `ranks`
    bands, else target (interleaved bands balance the per-rank work)."""
    for br in range(target, height + 1):
        if height % br == 0 and (height // br) % ranks == 0:
            return br
    return target


def global_rows(height, band_rows, rank, ranks):
    """Global row index of every local row of rank's buffer (-1 for padding)."""
    out = []
    for b in bands_of_rank(height, band_rows, rank, ranks):
        for r in range(band_rows):
            y = b * band_rows + r
            out.append(y if y < height else -1)
    return out


def unshuffle(gathered, height, band_rows, ranks):
    """numpy reference of frm_unshuffle_bands: gathered = [ranks, buffer_rows, W, 4]."""
    w = gathered.shape[2]
    out = np.zeros((height, w, 4), dtype=gathered.dtype)
    for y in range(height):
        b, r = divmod(y, band_rows)
        rank, j = b % ranks, b // ranks
        out[y] = gathered[rank, j * band_rows + r]
    return out
