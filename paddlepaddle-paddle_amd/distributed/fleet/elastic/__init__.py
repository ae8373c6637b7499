"""paddle.distributed.fleet.elastic (reference: fleet/elastic/__init__.py, manager.py).

The membership service is ``distributed/elastic.py`` (TCPStore registry); the launcher drives
it (``python -m paddle.distributed.launch --elastic_server host:port --np MIN:MAX``)."""
from ...elastic import ElasticManager, ElasticStatus, ElasticLevel, parse_np, connect_store  # noqa: F401


def enable_elastic(args, distribute_mode=None):
    return bool(getattr(args, 'elastic_server', None) or __import__('os').environ.get('PADDLE_ELASTIC_SERVER'))


def launch_elastic(args, distribute_mode=None):
    from ...launch import launch
    argv = ['--elastic_server', args.elastic_server, '--np', str(args.np), '--job_id', getattr(args, 'job_id', 'default')]
    return launch(argv + [args.training_script] + list(getattr(args, 'training_script_args', [])))
