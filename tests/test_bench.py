"""bench.py's driver contract on the CPU: ``--gpus N`` without a launcher starts N rank
processes by itself (the driver's scaling run must not measure one GPU), with a rendezvous on
127.0.0.1; ``--dry-launch`` reports them without starting anything."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    env.update(env_extra or {})
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=env, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_gpus_n_starts_n_ranks():
    plan = _run(['--gpus', '2', '--dry-launch', '--steps', '3'])
    assert plan['launch'] == 'self' and plan['ranks'] == 2
    assert [e['RANK'] for e in plan['env']] == ['0', '1'] and {e['WORLD_SIZE'] for e in plan['env']} == {'2'}
    assert {e['MASTER_ADDR'] for e in plan['env']} == {'127.0.0.1'} and len({e['MASTER_PORT'] for e in plan['env']}) == 1
    for cmd in plan['commands']:
        assert cmd[1].endswith('bench.py') and '--dry-launch' not in cmd and cmd[-2:] == ['--steps', '3']


def test_launcher_present_means_no_self_launch():
    plan = _run(['--gpus', '4', '--dry-launch'], {'WORLD_SIZE': '4'})
    assert plan == {'launch': 'none', 'ranks': 4}
    assert _run(['--dry-launch'])['ranks'] == 1
