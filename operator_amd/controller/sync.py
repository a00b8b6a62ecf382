"""Pattern repository sync: Git -> local pattern cache (J/service/PatternSyncService.java).

* clone (branch default ``main``) or pull into ``<cache>/<library>/<repo>`` (:42-77);
* HTTPS credentials ``user:pass`` or a bare token (empty user) (:139-152);
  passed to git as an ``http.extraHeader`` so they never land in .git/config;
* counts *.yaml / *.yml after sync (:228-253); available libraries are the
  YAML basenames under ``<cache>/<library>`` (:88-114);
* the cache root is configurable (Q10: the reference hard-codes /shared/patterns
  and ignores ``pattern.cache.directory``).

Implemented with the ``git`` CLI (JGit is a Java library); tests use local
bare repositories, since there is no network.
"""
from __future__ import annotations

import base64
import logging
import os
import subprocess
from pathlib import Path

log = logging.getLogger(__name__)


class SyncError(RuntimeError):
    pass


def _auth_args(credentials: str | None) -> list[str]:
    if not credentials or not credentials.strip():
        return []
    parts = credentials.split(":", 1)
    user, pw = (parts[0], parts[1]) if len(parts) == 2 else ("", credentials)
    tok = base64.b64encode(f"{user}:{pw}".encode()).decode()
    return ["-c", f"http.extraHeader=Authorization: Basic {tok}"]


def _git(args: list[str], cwd: str | None = None, timeout: float = 300.0) -> str:
    env = dict(os.environ, GIT_TERMINAL_PROMPT="0")
    r = subprocess.run(["git", *args], cwd=cwd, capture_output=True, text=True, timeout=timeout, env=env)
    if r.returncode != 0:
        raise SyncError(f"git {' '.join(a for a in args if 'Authorization' not in a)} failed: "
                        f"{r.stderr.strip() or r.stdout.strip()}")
    return r.stdout


def yaml_files(root: Path) -> list[Path]:
    if not root.exists():
        return []
    out = [p for p in root.rglob("*") if p.is_file() and p.suffix in (".yaml", ".yml") and ".git" not in p.parts]
    return sorted(out)


class PatternSync:
    def __init__(self, cache_dir: str | os.PathLike):
        self.cache_dir = Path(cache_dir)

    def repo_path(self, library: str, repo_name: str) -> Path:
        return self.cache_dir / library / repo_name

    def sync_repository(self, library: str, repo: dict, credentials: str | None = None) -> str:
        """Clone or pull; returns the HEAD commit."""
        name, url = repo.get("name"), repo.get("url")
        if not name or not url:
            raise SyncError("repository name and url are required")
        branch = repo.get("branch") or "main"
        lib_path = self.cache_dir / library
        lib_path.mkdir(parents=True, exist_ok=True)
        path = lib_path / name
        auth = _auth_args(credentials)
        try:
            if (path / ".git").exists():
                log.info("Pulling latest changes for repository at %s", path)
                _git([*auth, "fetch", "--depth", "1", "origin", branch], cwd=str(path))
                _git(["checkout", "-q", "-B", branch, "FETCH_HEAD"], cwd=str(path))
            else:
                log.info("Cloning repository %s to %s", url, path)
                _git([*auth, "clone", "-q", "--depth", "1", "--branch", branch, url, str(path)])
        except SyncError as e:
            raise SyncError(f"Repository sync failed: {e}") from e
        n = len(yaml_files(path))
        if n == 0:
            log.warning("No YAML pattern files found in repository at %s", path)
        else:
            log.info("Found %d YAML pattern files in repository at %s", n, path)
        return _git(["rev-parse", "HEAD"], cwd=str(path)).strip()

    def available_libraries(self, library: str) -> list[str]:
        out = []
        for p in yaml_files(self.cache_dir / library):
            out.append(p.name[: -len(p.suffix)])
        return out

    def yaml_count(self) -> int:
        return len(yaml_files(self.cache_dir))
