"""nn/utils/misc.py of the reference: log formatting, model registry, code zip."""
import inspect
import os
import zipfile

import numpy as np


def log_metrics(logger, prefix, metrics):
    metrics_string = " ".join([k + "=%s" % metrics[k] for k in sorted(metrics.keys())])
    logger.info(prefix + " " + metrics_string)


def classes_in_module(module):
    classes = {}
    for name, obj in inspect.getmembers(module):
        if inspect.isclass(obj) and obj.__module__ == module.__name__:
            classes[name] = obj
    return classes


def rgb2gray(rgb):
    return np.dot(rgb[..., :3], [0.299, 0.587, 0.114])


def zipdir(path, save_dir):
    """Snapshot the .py sources into save_dir/code.zip (misc.py:22-32)."""
    with zipfile.ZipFile(os.path.join(save_dir, 'code.zip'), 'w', zipfile.ZIP_DEFLATED) as zipf:
        for root, dirs, files in os.walk(path):
            dirs[:] = [d for d in dirs if d not in ("__pycache__", ".git", "build")]
            for file in files:
                if file.endswith(".py"):
                    zipf.write(os.path.join(root, file),
                               os.path.relpath(os.path.join(root, file), os.path.join(path, '..')))
