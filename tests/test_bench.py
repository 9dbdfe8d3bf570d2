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


def test_rank_bookkeeping_keeps_stdout_clean(tmp_path):
    """Two gloo ranks through bench._Comm (barrier, max, sum, the unique-id broadcast): nothing
    reaches stdout but what rank 0 prints -- gloo announces its peers on stdout, which would
    break the driver's one-JSON-line contract."""
    script = tmp_path / 'ranks.py'
    script.write_text(
        'import json, os, sys\n'
        'sys.path.insert(0, %r)\n'
        'import bench\n'
        'c = bench._Comm(2)\n'
        'r = int(os.environ["RANK"])\n'
        'm = c.max(r + 1.5); s = c.sum(r + 1); b = c.broadcast_bytes(b"id" if r == 0 else None)\n'
        'c.barrier(); c.close()\n'
        'if r == 0: print(json.dumps([m, s, b.decode()]))\n' % ROOT)
    import socket
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE='2', RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-500:] for o in outs]
    assert json.loads(outs[0][0]) == [2.5, 3, 'id'] and outs[0][0].count('\n') == 1, outs[0][0]
    assert outs[1][0] == ''


def _hang_script(tmp_path, timeout_s=2.0):
    """Two gloo ranks through bench._run_c5_guarded with a c5 that never returns on rank 1
    (a hung collective) and waits for it on rank 0."""
    script = tmp_path / 'hang.py'
    script.write_text(
        'import json, os, sys, threading\n'
        'sys.path.insert(0, %r)\n'
        'import bench\n'
        'r = int(os.environ["RANK"])\n'
        'c = bench._Comm(2)\n'
        'def c5():\n'
        '    bench._stage("c5: timed steps: merge")\n'
        '    threading.Event().wait()  # blocks forever, like a collective whose peer never comes\n'
        'line = {"metric": "m", "value": 1.0, "c5": None}\n'
        'bench._run_c5_guarded(line, c5, c, r, 2, %r)\n'
        'print("not reached")\n' % (ROOT, timeout_s))
    return script


def test_hung_c5_fails_the_run_and_names_the_stage(tmp_path):
    """A c5 sub-record that hangs ends every rank with a non-zero status; rank 0 still prints
    the one JSON line, its c5.error carrying each rank's stage."""
    import socket
    script = _hang_script(tmp_path)
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE='2', RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    assert [p.returncode for p in procs] == [3, 3], [o[1][-800:] for o in outs]
    line = json.loads(outs[0][0].strip().splitlines()[-1])
    assert line['value'] == 1.0 and 'did not finish' in line['c5']['error']
    assert [s['rank'] for s in line['c5']['ranks']] == [0, 1]
    assert all(s['stage'] == 'c5: timed steps: merge' for s in line['c5']['ranks']), line['c5']
    assert 'not reached' not in outs[0][0] and outs[1][0] == ''


def test_launcher_reaps_the_ranks_when_one_fails(tmp_path):
    """The self-launcher returns the failing rank's status and terminates a rank that would
    otherwise never end (a peer stuck in a collective)."""
    sys.path.insert(0, ROOT)
    import time
    import bench
    plan = [([sys.executable, '-c', 'import time; time.sleep(600)'], {}),
            ([sys.executable, '-c', 'import sys; sys.exit(3)'], {})]
    t0 = time.monotonic()
    rc = bench._launch_ranks(2, [], False, plan=plan, grace_s=1.0)
    assert rc == 3 and time.monotonic() - t0 < 60
    ok = [([sys.executable, '-c', 'pass'], {}), ([sys.executable, '-c', 'pass'], {})]
    assert bench._launch_ranks(2, [], False, plan=ok) == 0
