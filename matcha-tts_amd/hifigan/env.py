"""AttrDict (hifigan/env.py:7-10): a dict whose keys are also attributes."""
import os
import shutil


class AttrDict(dict):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self


def build_env(config, config_name, path):
    target = os.path.join(path, config_name)
    if config != target:
        os.makedirs(path, exist_ok=True)
        shutil.copyfile(config, target)
