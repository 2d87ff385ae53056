"""mast3r_slam.config (config.py): the global config dict and its loaders."""
from monst3r_slam_amd.config import config, default_config, load_config  # noqa: F401


def set_global_config(cfg):
    """config.py: set_global_config — replace the process-wide config in place (the
    backend process receives the frontend's config this way)."""
    config.clear()
    config.update(cfg)
