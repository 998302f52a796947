"""jax.config stand-in: `from jax import config` and `from jax.config import config` both work."""


class _Config:
    def update(self, *a, **k):
        pass


config = _Config()
