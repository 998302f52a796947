"""Normalize -- the '-11' min/max wrapper of the reference (utils.py:1-33), host side."""
import numpy as np


class Normalize():
    def __init__(self, mn, mx, norm_type=None):
        self.mn = mn
        self.mx = mx
        if norm_type is None:
            norm_type = 'identity'
        if norm_type.lower() not in ['identity', '-11']:
            raise NotImplementedError('Only identity and -11 are implemented')
        self.norm_type = norm_type.lower()

    def fit(self, x):
        mn, mx = self.mn, self.mx
        if self.norm_type == '-11':
            return 2 * (x - mn) / (mx - mn) - 1
        return x

    def inverse(self, x):
        mn, mx = self.mn, self.mx
        if self.norm_type == '-11':
            return (x + 1) / 2 * (mx - mn) + mn
        return x

    def get_scale(self):
        mn, mx = self.mn, self.mx
        if self.norm_type == '-11':
            return 2 / (mx - mn)
        return 1

    def device_table(self, d):
        """[mn | (mx-mn) | 2/(mx-mn)] (3d doubles) as consumed by nngp_system.norm, or None."""
        if self.norm_type != '-11':
            return None
        mn = np.broadcast_to(np.asarray(self.mn, dtype=float), (d,))
        mx = np.broadcast_to(np.asarray(self.mx, dtype=float), (d,))
        return np.concatenate([mn, mx - mn, 2 / (mx - mn)])
