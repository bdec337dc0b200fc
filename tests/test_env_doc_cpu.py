"""docs/ENV.md lists every CAKE_* environment variable the package, the native sources and
bench.py read (a knob nobody can find is a knob nobody can set)."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
READ = re.compile(r'(?:getenv\("|environ\.get\("|environ\["|environ\.get\(\')(CAKE_[A-Z0-9_]+)')


def test_every_env_var_is_documented():
    used = set()
    files = [ROOT / "bench.py", *ROOT.joinpath("cake_amd").rglob("*.py")]
    files += [p for ext in ("*.cpp", "*.h", "*.hip") for p in ROOT.joinpath("cake_amd").rglob(ext)]
    for p in files:
        used |= set(READ.findall(p.read_text(errors="replace")))
    doc = (ROOT / "docs" / "ENV.md").read_text()
    missing = sorted(v for v in used if f"`{v}" not in doc)
    assert not missing, f"undocumented environment variables: {missing}"
