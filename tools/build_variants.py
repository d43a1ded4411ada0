"""Build A/B variants of libmz (muzero.jl_amd/lib/libmz_<name>.so) from the
current sources with extra compile flags, or from a git revision's sources:
  python tools/build_variants.py name=-DFLAG,... [rev:name=<git rev>] ..."""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _mzpkg  # noqa: E402

_mzpkg.load()
from muzero_jl_amd import build as b  # noqa: E402

lib = os.path.join(ROOT, "muzero.jl_amd", "lib")
for arg in sys.argv[1:]:
    if arg.startswith("rev:"):
        name, rev = arg[4:].split("=", 1)
        tmp = tempfile.mkdtemp()
        subprocess.run(f"git -C {ROOT} archive {rev} muzero.jl_amd include | tar -x -C {tmp}", shell=True, check=True)
        src = os.path.join(tmp, "muzero.jl_amd", "build.py")
        env = dict(os.environ)
        code = (f"import importlib.util,sys,types;"
                f"pkg=types.ModuleType('v');pkg.PKG_DIR={os.path.join(tmp, 'muzero.jl_amd')!r};"
                f"pkg.LIB_PATH={os.path.join(tmp, 'lib', 'libmz.so')!r};sys.modules['v']=pkg;"
                f"spec=importlib.util.spec_from_file_location('v.build',{src!r});m=importlib.util.module_from_spec(spec);"
                f"m.__package__='v';spec.loader.exec_module(m);m.build(force=True)")
        subprocess.run([sys.executable, "-c", code], check=True, env=env)
        os.replace(os.path.join(tmp, "lib", "libmz.so"), os.path.join(lib, f"libmz_{name}.so"))
    else:
        name, flags = arg.split("=", 1)
        extra = [f for f in flags.split(",") if f]
        b.build(force=True, out=os.path.join(lib, f"libmz_{name}.so"), objdir=os.path.join(lib, f"obj_{name}"),
                extra=extra)
    print("built", name, flush=True)
