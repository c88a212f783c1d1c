"""Job staging: the local replacement for Docker image build + push.

Reference ``TFC/core/containerize.py`` tarred the entry-point directory,
generated a Dockerfile and built/pushed an image.  On an MI355X node the
"image" is a job directory::

    <jobs_root>/<job_id>/
        app/                 <- entry-point directory tree (same file map as the reference:
                                entry dir -> app/, wrapper -> app/<wrapper>, requirements -> app/)
        manifest.json        <- the Dockerfile equivalent: python, entry, env, requirements,
                                framework/ROCm/arch stamp
        logs/                <- per-rank logs (filled by the launcher)
        job.json             <- job metadata + exit codes (launcher)

Requirements are installed best-effort with ``pip install --user`` only when
``CLOUD_AMD_PIP_INSTALL=1`` (GPU boxes have no package index).

Staging is part of ``run()`` -> first-step latency, so it stays cheap:

* **code** files of the entry directory (``.py``, ``.ipynb``, built extensions ``.so`` and
  native sources) are *hard-linked* into ``app/``; **every other file is copied**.  Ranks
  run with ``cwd=app``, so a job that rewrites a file it finds there (``model.h5``, a
  checkpoint, a CSV log, opened ``"w"`` or ``"a"``) writes its own copy and never the
  user's tree, and two jobs staged from one directory never share a writable file -- the
  isolation of the reference's tarball (``containerize.py:124-132``) at the cost of
  copying data files only.  ``CLOUD_AMD_STAGE_COPY=1`` copies code too (a source edited
  in place while its job runs is then invisible to the job);
* VCS / cache directories and ``jobs/`` are skipped; project-specific excludes come from
  a ``.cloudamdignore`` file at the top of the entry directory (one ``fnmatch`` pattern
  per line, ``#`` comments), so a user package named ``build/`` or ``profiles/`` ships
  unless the project says otherwise;
* the framework stamp reads package metadata and never imports torch (a cold
  ``import torch`` costs ~2 s in the launching process, which never needs it).
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import time

from ..version import ARCH, __version__

IGNORE = shutil.ignore_patterns("__pycache__", "*.pyc", ".git", "jobs", ".ipynb_checkpoints", ".pytest_cache",
                                ".hypothesis")
IGNORE_FILE = ".cloudamdignore"
# hard-linked (read by the job, never written by it); everything else is copied
LINK_SUFFIXES = (".py", ".pyi", ".ipynb", ".so", ".hip", ".h", ".hpp", ".cpp", ".cc", ".c")


def _user_ignores(src_dir):
    path = os.path.join(src_dir, IGNORE_FILE)
    if not os.path.isfile(path):
        return ()
    with open(path) as f:
        return tuple(ln.strip().rstrip("/") for ln in f if ln.strip() and not ln.lstrip().startswith("#"))


def _ignore(root, src_dir=None):
    root = os.path.abspath(root)
    extra = shutil.ignore_patterns(*_user_ignores(src_dir)) if src_dir else None

    def ign(d, names):
        out = set(IGNORE(d, names))
        if extra is not None:
            out.update(extra(d, names))
        out.update(n for n in names if os.path.abspath(os.path.join(d, n)) == root)
        return out

    return ign


def jobs_root():
    return os.path.abspath(os.environ.get("CLOUD_AMD_JOBS_DIR", os.path.join(os.getcwd(), "jobs")))


def file_path_map(entry_point, preprocessed_entry_point, requirements_txt=None, destination_dir="app"):
    """source path -> path relative to the job dir (reference containerize.py:235-277)."""
    if entry_point is None:
        entry_point = sys.argv[0]
    entry_dir = os.path.dirname(os.path.abspath(entry_point)) if entry_point else os.getcwd()
    m = {entry_dir: destination_dir}
    if preprocessed_entry_point is not None:
        m[preprocessed_entry_point] = os.path.join(destination_dir, os.path.basename(preprocessed_entry_point))
    if requirements_txt is not None:
        m[os.path.abspath(requirements_txt)] = os.path.join(destination_dir, os.path.basename(requirements_txt))
    return m


def _framework_stamp():
    """cloud_amd / torch / HIP / arch versions from package metadata and torch's generated
    ``version.py`` text -- without importing torch."""
    stamp = {"cloud_amd": __version__, "arch": ARCH, "python": sys.version.split()[0]}
    try:
        import importlib.metadata as md

        stamp["torch"] = md.version("torch")
    except Exception:  # pragma: no cover - torch not installed
        return stamp
    try:
        import importlib.util
        import re

        spec = importlib.util.find_spec("torch")  # locates the package, does not import it
        if spec is not None and spec.submodule_search_locations:
            vfile = os.path.join(list(spec.submodule_search_locations)[0], "version.py")
            with open(vfile) as f:
                m = re.search(r"^hip\s*(?::\s*[^=]+)?=\s*['\"]([^'\"]+)['\"]", f.read(), re.M)
            stamp["hip"] = m.group(1) if m else None
    except Exception:  # pragma: no cover
        pass
    return stamp


def _link_or_copy(src, dst):
    """Hard link (cheap, same filesystem); fall back to a copy."""
    try:
        os.link(src, dst)
    except OSError:
        shutil.copy2(src, dst)
    return dst


def _stage_file(src, dst):
    """Code is hard-linked, data copied (``CLOUD_AMD_STAGE_COPY=1``: everything copied)."""
    if os.environ.get("CLOUD_AMD_STAGE_COPY") != "1" and src.endswith(LINK_SUFFIXES):
        return _link_or_copy(src, dst)
    return shutil.copy2(src, dst)


def stage_job(job_id, entry_point, preprocessed_entry_point, requirements_txt=None, entry_point_args=None,
              env=None, root=None):
    """Create the job directory; return (job_dir, run_target) where run_target is the script to exec."""
    root = root or jobs_root()
    job_dir = os.path.join(root, job_id)
    app = os.path.join(job_dir, "app")
    os.makedirs(os.path.join(job_dir, "logs"), exist_ok=True)
    fmap = file_path_map(entry_point, preprocessed_entry_point, requirements_txt)
    for src, rel in fmap.items():
        dst = os.path.join(job_dir, rel)
        if os.path.isdir(src):
            if os.path.abspath(src).startswith(os.path.abspath(job_dir)):
                raise ValueError("entry-point directory is inside the job directory")
            shutil.copytree(src, dst, ignore=_ignore(root, src), dirs_exist_ok=True, symlinks=False,
                            copy_function=_stage_file)
        else:
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            if os.path.exists(dst):
                if os.path.samefile(src, dst):  # already linked in with the entry directory
                    continue
                os.remove(dst)
            _stage_file(src, dst)
    if preprocessed_entry_point is not None:
        target = os.path.join(app, os.path.basename(preprocessed_entry_point))
    else:
        target = os.path.join(app, os.path.basename(entry_point or sys.argv[0]))
    manifest = {
        "job_id": job_id,
        "created": time.time(),
        "entrypoint": ["python", os.path.relpath(target, job_dir)] + list(entry_point_args or []),
        "workdir": "app",
        "requirements": os.path.basename(requirements_txt) if requirements_txt else None,
        "env": dict(env or {}),
        "framework": _framework_stamp(),
        "file_map": {k: v for k, v in fmap.items()},
    }
    with open(os.path.join(job_dir, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=2)
    if requirements_txt and os.environ.get("CLOUD_AMD_PIP_INSTALL") == "1":
        subprocess.run([sys.executable, "-m", "pip", "install", "--user", "-r",
                        os.path.join(app, os.path.basename(requirements_txt))], check=False)
    return job_dir, target
