"""paddle.distributed.fleet.utils (reference: python/paddle/distributed/fleet/utils/__init__.py)."""
from ..recompute import recompute  # noqa: F401
from . import sequence_parallel_utils  # noqa: F401
from .hybrid_parallel_util import fused_allreduce_gradients, broadcast_mp_parameters, broadcast_dp_parameters  # noqa: F401


class LocalFS:
    """Minimal local filesystem helper (reference fleet.utils.LocalFS)."""

    def mkdirs(self, p):
        import os
        os.makedirs(p, exist_ok=True)

    def is_exist(self, p):
        import os
        return os.path.exists(p)

    def ls_dir(self, p):
        import os
        ents = os.listdir(p)
        return [e for e in ents if os.path.isdir(os.path.join(p, e))], \
               [e for e in ents if os.path.isfile(os.path.join(p, e))]

    def delete(self, p):
        import shutil
        import os
        shutil.rmtree(p) if os.path.isdir(p) else (os.remove(p) if os.path.exists(p) else None)


class ExecuteError(RuntimeError):
    pass


class HDFSClient:
    """HDFS access through the ``hadoop fs`` command line (reference fleet/utils/fs.py HDFSClient):
    same method surface as LocalFS.  ``hadoop_home`` must hold bin/hadoop; ``configs`` become
    ``-D key=value`` options.  No client is bundled: a missing binary raises ExecuteError."""

    def __init__(self, hadoop_home, configs=None, time_out=5 * 60 * 1000, sleep_inter=1000):
        import os
        self._bin = os.path.join(hadoop_home, 'bin', 'hadoop')
        self._opts = []
        for k, v in (configs or {}).items():
            self._opts += ['-D', f'{k}={v}']
        self._timeout = time_out / 1000.0

    def _run(self, *args, check=True):
        import os
        import subprocess
        if not os.path.exists(self._bin):
            raise ExecuteError(f"hadoop client not found at {self._bin}")
        r = subprocess.run([self._bin, 'fs', *self._opts, *args], capture_output=True, text=True,
                           timeout=self._timeout)
        if check and r.returncode != 0:
            raise ExecuteError(f"hadoop fs {' '.join(args)} failed: {r.stderr.strip()}")
        return r

    def is_exist(self, fs_path):
        return self._run('-test', '-e', fs_path, check=False).returncode == 0

    def is_dir(self, fs_path):
        return self._run('-test', '-d', fs_path, check=False).returncode == 0

    def is_file(self, fs_path):
        return self.is_exist(fs_path) and not self.is_dir(fs_path)

    def ls_dir(self, fs_path):
        dirs, files = [], []
        for line in self._run('-ls', fs_path).stdout.splitlines():
            parts = line.split()
            if len(parts) < 8:
                continue
            name = parts[-1].rstrip('/').split('/')[-1]
            (dirs if parts[0].startswith('d') else files).append(name)
        return dirs, files

    def mkdirs(self, fs_path):
        self._run('-mkdir', '-p', fs_path)

    def delete(self, fs_path):
        if self.is_exist(fs_path):
            self._run('-rm', '-r', fs_path)

    def upload(self, local_path, fs_path, multi_processes=1, overwrite=False):
        self._run('-put', *(['-f'] if overwrite else []), local_path, fs_path)

    def download(self, fs_path, local_path, multi_processes=1, overwrite=False):
        self._run('-get', *(['-f'] if overwrite else []), fs_path, local_path)

    def mv(self, fs_src_path, fs_dst_path, overwrite=False, test_exists=True):
        if overwrite and self.is_exist(fs_dst_path):
            self.delete(fs_dst_path)
        self._run('-mv', fs_src_path, fs_dst_path)

    def touch(self, fs_path, exist_ok=True):
        if self.is_exist(fs_path) and not exist_ok:
            raise FileExistsError(fs_path)
        self._run('-touchz', fs_path)

    def cat(self, fs_path=None):
        return self._run('-cat', fs_path).stdout.rstrip('\n')

    def need_upload_download(self):
        return True


class DistributedInfer:
    """Inference over a parameter-server-trained program (reference fleet/utils/ps_util.py): on
    the workers the sparse embedding tables stay on the servers (``distributed/ps`` pulls rows on
    lookup), so the distributed inference program is the main program itself once the worker is
    initialised."""

    def __init__(self, main_program=None, startup_program=None):
        from ....static import default_main_program, default_startup_program
        self.origin_main_program = main_program or default_main_program()
        self.origin_startup_program = startup_program or default_startup_program()
        self._inited = False

    def init_distributed_infer_env(self, exe, loss, role_maker=None, dirname=None):
        from .. import fleet
        if not fleet._inited:
            fleet.init(role_maker=role_maker, is_collective=False)
        if fleet.is_worker():
            fleet.init_worker()
        if dirname is not None:
            from ....static import load
            load(self.origin_main_program, dirname, exe)
        self._inited = True

    def get_dist_infer_program(self):
        return self.origin_main_program
