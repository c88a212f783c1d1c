"""Every CLOUD_AMD_* variable the code reads is declared (typed) in cloud_amd/config.py."""
import os
import re

from cloud_amd import config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_all_env_vars_declared():
    used = set()
    for base in ("cloud_amd", "bench", "examples", "csrc", "scripts"):
        for dp, dirs, files in os.walk(os.path.join(ROOT, base)):
            dirs[:] = [d for d in dirs if d != "old"]  # scripts/old: archived runs of removed switches
            for f in files:
                if f.endswith((".py", ".cpp", ".h", ".hip", ".sh")):
                    used |= set(re.findall(r"CLOUD_AMD_[A-Z0-9_]+", open(os.path.join(dp, f), errors="ignore").read()))
    used |= set(re.findall(r"CLOUD_AMD_[A-Z0-9_]+", open(os.path.join(ROOT, "bench.py")).read()))
    missing = sorted(u for u in used if u not in config.VARS)
    assert not missing, missing


def test_typed_parsing(monkeypatch):
    monkeypatch.setenv("CLOUD_AMD_BUCKET_MB", "32")
    monkeypatch.setenv("CLOUD_AMD_TRACE", "1")
    monkeypatch.delenv("CLOUD_AMD_GRAD_CHECK_EVERY", raising=False)
    assert config.get("CLOUD_AMD_BUCKET_MB") == 32.0
    assert config.get("CLOUD_AMD_TRACE") is True
    assert config.get("CLOUD_AMD_GRAD_CHECK_EVERY") == 0
    assert "CLOUD_AMD_COMM" in config.describe()
