"""Reference auto_parallel/process_mesh.py: ProcessMesh (defined in api.py)."""
from .api import ProcessMesh  # noqa: F401
