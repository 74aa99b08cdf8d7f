"""``ray_installed()`` (parity: ``p2pfl/utils/check_ray.py:26-42``) without the side effect of
starting Ray: True only if Ray imports and ``Settings.DISABLE_RAY`` is False."""

from myfyp_amd.settings import Settings


def ray_installed() -> bool:
    if Settings.DISABLE_RAY:
        return False
    try:
        import ray  # noqa: F401
    except ImportError:
        return False
    return True
