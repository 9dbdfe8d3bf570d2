"""Host-side logic that runs without a GPU: term normalisation, agg-spec parsing, wire
messages, bcolz layout, tar-of-tars gather, and the libbqgpu C ABI exports."""
import io
import os
import re
import tarfile
from collections import OrderedDict

import numpy as np
import pytest

from bqueryd_amd import _lib, bcolz_io, messages, rpc, terms, worker
from oracle import bquery_oracle as bo
from oracle import cbquery


# ---------------------------------------------------------------------------- where terms
@pytest.mark.parametrize('dtype', [np.bool_, np.int8, np.int16, np.int32, np.int64, np.uint8, np.uint16,
                                   np.uint32, np.uint64, np.float32, np.float64])
def test_term_normalisation_matches_oracle(dtype):
    values = [0, 1, -1, 2.5, -2.5, 3.0, 255, 256, -129, 2**31, 2**63, -2**63, 1e300, float('inf'),
              float('-inf'), float('nan'), True, False]
    for code in (1, 2, 5, 6, 7, 8):
        for v in values:
            got = terms.normalize(dtype, code, v)
            ref = cbquery.normalize_term(np.dtype(dtype), code, v)
            assert got[0] == ref[0], (dtype, code, v, got, ref)
            if got[0] not in (-1, 0):
                assert list(got[1]) == list(ref[1]) and list(got[2]) == list(ref[2]), (dtype, code, v)
    for members in ([1, 2, 3], [2.5, 3], [1000, 2, 2.0], [float('nan'), 1]):
        for code in (3, 4):
            got = terms.normalize(dtype, code, set(members))
            ref = cbquery.normalize_term(np.dtype(dtype), code, set(members))
            assert got[0] == ref[0], (dtype, code, members)


def test_term_parsing_errors():
    names = {'a': np.dtype(np.int32)}
    with pytest.raises(KeyError):
        terms.parse_terms(names, [('b', '==', 1)])
    with pytest.raises(KeyError):
        terms.parse_terms(names, [('a', 'like', 1)])
    with pytest.raises(ValueError):
        terms.parse_terms(names, [('a', 'in', 1)])
    with pytest.raises(ValueError):
        terms.parse_terms(names, [('a', 'nin', [])])
    assert terms.parse_terms(names, [('a', ' IN ', [4])]) == [('a', 1, 4)]
    assert terms.parse_terms(names, [('a', 'not in', (4,))]) == [('a', 2, 4)]


def test_agg_parsing_matches_oracle():
    dts = OrderedDict(a=np.dtype(np.int16), b=np.dtype(np.float32))
    cols = OrderedDict(a=np.zeros(1, np.int16), b=np.zeros(1, np.float32))
    spec = ['a', ['b', 'mean'], ['a', 'count', 'n'], ['b', 'sum', 's'], ['a', 'std', 'sd'],
            ['a', 'count_distinct', 'cd'], ['b', 'sorted_count_distinct', 'scd']]
    assert terms.parse_agg_list(dts, spec) == bo.parse_agg_list(cols, spec)
    with pytest.raises(NotImplementedError):
        terms.parse_agg_list(dts, [['a', 'median', 'm']])
    with pytest.raises(KeyError):
        terms.parse_agg_list(dts, [['z', 'sum', 'z']])


# ---------------------------------------------------------------------------- wire format
# A Python-2 cPickle (protocol 0) of the params the reference RPC sends for
# rpc.groupby(['f.bcolzs'], ['payment_type'], [['fare_amount', 'sum', 'fare_amount']], [],
# aggregate=True) (rpc.py:88-96), base64-encoded as str.encode('base64') does.
PY2_PARAMS = (b"(dp1\nS'args'\np2\n((lp3\nS'f.bcolzs'\np4\na(lp5\nS'payment_type'\np6\na(lp7\n(lp8\n"
              b"S'fare_amount'\np9\naS'sum'\np10\nag9\naa(lp11\ntp12\nsS'kwargs'\np13\n(dp14\n"
              b"S'aggregate'\np15\nI01\nss.")


def test_py2_params_decode():
    import base64
    msg = messages.msg_factory({'msg_type': 'calc', 'payload': 'groupby',
                                'params': base64.encodebytes(PY2_PARAMS).decode('ascii')})
    assert isinstance(msg, messages.CalcMessage)
    args, kwargs = msg.get_args_kwargs()
    assert args == (['f.bcolzs'], ['payment_type'], [['fare_amount', 'sum', 'fare_amount']], [])
    assert kwargs == {'aggregate': True}


def test_message_roundtrip():
    m = messages.RPCMessage({'payload': 'groupby'})
    m.set_args_kwargs(['a.bcolz', ['k'], [['v', 'sum', 'v']], [('k', '>', 1)]], {'aggregate': True})
    js = m.to_json()
    m2 = messages.msg_factory(js)
    assert isinstance(m2, messages.RPCMessage) and m2.isa('groupby') and m2.isa(messages.RPCMessage())
    args, kwargs = m2.get_args_kwargs()
    assert args[0] == 'a.bcolz' and kwargs == {'aggregate': True}
    assert '\n' in m['params']  # MIME base64 like str.encode('base64')
    assert isinstance(messages.msg_factory('not json'), messages.Message)


# ---------------------------------------------------------------------------- bcolz / tar
def test_bcolz_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    cols = OrderedDict(a=rng.integers(-9, 9, 300_001).astype(np.int8), b=rng.normal(size=300_001),
                       c=np.arange(300_001, dtype=np.uint64), d=rng.random(300_001) < 0.5,
                       e=np.zeros(300_001, np.float32))
    root = str(tmp_path / 's.bcolz')
    bcolz_io.write_ctable(root, cols, chunklen=65536)
    assert bcolz_io.ctable_names(root) == list(cols)
    assert bcolz_io.ctable_len(root) == 300_001
    back = bcolz_io.read_ctable(root)
    for k in cols:
        assert back[k].dtype == cols[k].dtype
        np.testing.assert_array_equal(back[k], cols[k])
    # chunk files carry the 16-byte bloscpack header + one blosc frame
    with open(os.path.join(root, 'b', 'data', '__0.blp'), 'rb') as f:
        head = f.read(16)
    assert head[:4] == b'blpk' and int.from_bytes(head[8:16], 'little', signed=True) == 1
    assert len(os.listdir(os.path.join(root, 'b', 'data'))) == 5  # 4 full chunks + leftover


def test_tar_of_tars_and_concat_merge(tmp_path):
    tables = []
    results = OrderedDict()
    for i in range(3):
        t = OrderedDict(k=np.array([i, i + 1], np.int32), s=np.array([1.5, 2.5]) * i)
        d = str(tmp_path / ('result_%d' % i))
        bcolz_io.write_ctable(d, t)
        results['shard_%d.bcolzs' % i] = worker.tar_directory(d)
        tables.append(t)
    results['empty.bcolzs'] = ''
    blob = rpc.tar_of_tars(results)
    with tarfile.open(fileobj=io.BytesIO(blob)) as tf:
        assert sorted(m.name for m in tf.getmembers()) == ['shard_%d.bcolzs' % i for i in range(3)]
        inner = tarfile.open(fileobj=io.BytesIO(tf.extractfile('shard_0.bcolzs').read()))
        assert inner.getnames()[0] == 'result_0'
    back = rpc.read_shard_results(blob)
    merged = rpc.merge_tables(back, ['k'], [['s', 'sum', 's']], aggregate=False)
    ref = bo.client_merge(tables, ['k'], [['s', 'sum', 's']], aggregate=False)
    for c in ref:
        np.testing.assert_array_equal(merged[c], ref[c])
    assert rpc.merge_tables([], ['k'], [], aggregate=True) is None


@pytest.mark.parametrize('nrows', [0, 1, 70_000, 600_000])
def test_ctable_tar_matches_tar_of_written_ctable(tmp_path, nrows, monkeypatch):
    """The in-memory result tar has the members, order and contents of tarfile.add over the
    ctable directory write_ctable creates (worker.py:335-346) -- also for a zero-row result,
    whose columns have no chunk file but keep their data/ and meta/ directories; 600 K rows
    take the compression pool (several chunks per column, frames in one reused arena)."""
    rng = np.random.default_rng(nrows)
    cols = OrderedDict(k=rng.integers(0, 9, nrows).astype(np.int32), s=rng.normal(size=nrows),
                       n=np.arange(nrows, dtype=np.int64))
    d = str(tmp_path / 'result_abcdefgh')
    bcolz_io.write_ctable(d, cols)
    ref = worker.tar_directory(d)
    import time as _time
    monkeypatch.setattr(_time, 'time', lambda: 1_700_000_000.25)
    got = bcolz_io.ctable_tar(cols, 'result_abcdefgh')
    assert bcolz_io.ctable_tar(cols, 'result_abcdefgh') == got  # the reused arena
    with tarfile.open(fileobj=io.BytesIO(ref)) as a, tarfile.open(fileobj=io.BytesIO(got)) as b:
        ma, mb = a.getmembers(), b.getmembers()
        assert [(m.name, m.isdir()) for m in ma] == [(m.name, m.isdir()) for m in mb]
        for x, y in zip(ma, mb):
            if x.isfile():
                assert a.extractfile(x).read() == b.extractfile(y).read(), x.name
    assert 'result_abcdefgh/k/data' in [m.name for m in mb]
    back = rpc.read_shard_results(rpc.tar_of_tars(OrderedDict([('f.bcolzs', got)])))
    assert len(back) == 1
    for c in cols:
        np.testing.assert_array_equal(back[0][c], cols[c])


def test_node_message_routing_pins_the_gpu_worker():
    """The node-level message is pinned to the GPU calc worker that holds ALL of its files,
    so handle_out (controller.py:248-257) cannot hand it to another worker that holds only the
    first file; replicated files on a CPU worker keep their per-file path."""
    import random
    files = ['f%d.bcolzs' % i for i in range(6)]
    spec = [files, ['k'], [['s', 'sum', 's']], []]
    workers = {
        'cpu0': {'workertype': 'calc', 'node': 'n0'},            # holds f0 (and f5) too
        'dl0': {'workertype': 'download', 'node': 'n1'},
        'gpuA': {'workertype': 'calc', 'node': 'n1', 'gpu_node': True},
        'gpuB': {'workertype': 'calc', 'node': 'n2', 'gpu_node': True},  # holds only f4
    }
    fmap = {'f0.bcolzs': {'cpu0', 'gpuA'}, 'f1.bcolzs': {'gpuA'}, 'f2.bcolzs': {'gpuA', 'dl0'},
            'f3.bcolzs': {'gpuA'}, 'f4.bcolzs': {'gpuB'}, 'f5.bcolzs': {'cpu0'}}
    out = rpc.fan_out(spec, {'aggregate': True}, workers, fmap)
    node = [m for m in out if isinstance(m['args'][0], list)]
    assert len(node) == 1 and node[0]['worker_id'] == 'gpuA'
    assert node[0]['args'][0] == files[:4] and node[0]['filename'] == 'f0.bcolzs'
    per_file = [m for m in out if not isinstance(m['args'][0], list)]
    assert [m['filename'] for m in per_file] == ['f4.bcolzs', 'f5.bcolzs']  # gpuB holds one file only
    for seed in range(50):
        rng = random.Random(seed)
        # pinned: whichever workers are free, the node message goes to gpuA
        assert rpc.route(node[0], workers, fmap, rng=rng) == 'gpuA'
        # an unpinned message for f0 (the pre-patch behaviour) may reach cpu0 -- the bug the pin fixes
        assert rpc.route({'filename': 'f0.bcolzs', 'worker_id': None}, workers, fmap, rng=rng) in ('cpu0', 'gpuA')
        assert rpc.route(per_file[0], workers, fmap, rng=rng) == 'gpuB'
        assert rpc.route(per_file[1], workers, fmap, rng=rng) == 'cpu0'
    seen = {rpc.route({'filename': 'f0.bcolzs', 'worker_id': None}, workers, fmap, rng=random.Random(s))
            for s in range(50)}
    assert seen == {'cpu0', 'gpuA'}
    # busy workers are skipped by find_free_worker (controller.py:123-124); needs_local keeps the node
    busy = dict(workers, cpu0=dict(workers['cpu0'], busy=True))
    assert rpc.route({'filename': 'f5.bcolzs', 'worker_id': None}, busy, fmap) is None
    assert rpc.route({'filename': 'f1.bcolzs', 'worker_id': '__needs_local__'}, workers, fmap, node_name='n1') == 'gpuA'
    assert rpc.route({'filename': 'f1.bcolzs', 'worker_id': '__needs_local__'}, workers, fmap, node_name='n0') is None
    # a GPU worker never gets a node message for files it does not hold: no files -> per-file only
    assert all(m['worker_id'] is None for m in rpc.fan_out([['f5.bcolzs', 'f4.bcolzs'], ['k'], [], []],
                                                           {'aggregate': True}, workers, fmap))


def test_fan_out_and_gather_accounting(tmp_path):
    """controller.py:471-508 scatter and 146-221 gather, with the node-level patch: the RPC
    completes only when every file is covered, by its own reply or by a node reply."""
    files = ['f%d.bcolzs' % i for i in range(5)]
    spec = [files, ['k'], [['s', 'sum', 's']], []]
    workers = {'gpu0': {'gpu_node': True, 'workertype': 'calc'}, 'gpu1': {'gpu_node': True, 'workertype': 'calc'}}
    fmap = {f: {'gpu0'} for f in files[:3]}
    fmap['other.bcolzs'] = {'gpu1'}
    # without aggregate=True (or without GPU nodes) every file gets its own message
    assert [m['args'][0] for m in rpc.fan_out(spec, {})] == files
    assert [m['args'][0] for m in rpc.fan_out(spec, {'aggregate': False}, workers, fmap)] == files
    out = rpc.fan_out(spec, {'aggregate': True}, workers, fmap)
    assert out[0]['args'][0] == files[:3] and out[0]['worker_id'] == 'gpu0'
    assert [m['args'][0] for m in out[1:]] == files[3:] and all(m['worker_id'] is None for m in out[1:])
    assert all(m['args'][1:] == spec[1:] for m in out)
    msgs = [m['args'] for m in out]
    with pytest.raises(ValueError):
        rpc.fan_out([[], ['k'], [], []], {})
    tables = []
    for i in range(3):
        t = OrderedDict(k=np.array([i, 7], np.int32), s=np.array([1.0, 2.0]))
        tables.append(t)
    seg = rpc.CalcSegment(files)
    assert not seg.add_reply(msgs[1], bcolz_io.ctable_tar(tables[1], 'result_a'))
    with pytest.raises(RuntimeError):
        seg.tar()
    assert not seg.add_reply(msgs[2], '')  # factorization-check early-out: no member
    with pytest.raises(KeyError):
        seg.add_reply([['nope.bcolzs']] + spec[1:], b'x')
    assert seg.add_reply(msgs[0], bcolz_io.ctable_tar(tables[0], 'result_b'))  # covers f0..f2
    back = rpc.read_shard_results(seg.tar())
    assert len(back) == 2
    got = bo.client_merge(back, ['k'], [['s', 'sum', 's']], aggregate=True)
    ref = bo.client_merge([tables[0], tables[1]], ['k'], [['s', 'sum', 's']], aggregate=True)
    for c in ref:
        np.testing.assert_array_equal(np.sort(got[c]), np.sort(ref[c]))


# ---------------------------------------------------------------------------- C ABI
def test_library_exports_every_declared_symbol():
    header = open(os.path.join(os.path.dirname(__file__), '..', 'include', 'bqgpu.h')).read()
    declared = sorted(set(re.findall(r'^\s*(?:const\s+)?\w[\w\s\*]*?\b(bqg_\w+)\s*\(', header, re.M)))
    assert len(declared) >= 25, declared
    lib = _lib.lib()
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_lib._PROTOS), set(declared) ^ set(_lib._PROTOS)
    assert lib.bqg_abi_version() == _lib.ABI_VERSION == 10


def test_library_fails_loudly_without_gpu():
    if os.path.exists('/dev/kfd'):
        pytest.skip('a GPU is present')
    from bqueryd_amd.engine import Device
    with pytest.raises(_lib.BqgError):
        Device(0)


def test_groupby_plan_cache_key_is_exact():
    """ShardTable caches the parsed query per query text; numpy-array term values (whose repr
    is abbreviated) are never cached, and a different value list is a different plan."""
    import numpy as np
    from bqueryd_amd.engine import ShardTable

    class Fake(ShardTable):
        def __init__(self):  # no device: only the host-side planning is exercised
            self.dtypes = {'a': np.dtype(np.int32), 'b': np.dtype(np.float64)}
            self._slot = {'a': 0, 'b': 1}

    t = Fake()
    p1 = t._plan(['a'], [['b', 'sum', 's']], [('a', 'in', [1, 2])], None)
    p2 = t._plan(['a'], [['b', 'sum', 's']], [('a', 'in', [1, 2])], None)
    p3 = t._plan(['a'], [['b', 'sum', 's']], [('a', 'in', [1, 3])], None)
    assert p1[2] is p2[2] and p3[2] is not p1[2]
    big = list(range(5000))
    big2 = list(big)
    big2[2500] = -1
    q1 = t._plan(['a'], [['b', 'sum', 's']], [('a', 'in', big)], None)
    q2 = t._plan(['a'], [['b', 'sum', 's']], [('a', 'in', big2)], None)
    assert q1[2] is not q2[2]
    assert len(t._plans) == 4
    with pytest.raises(ValueError):  # bquery: `in` takes lists, sets or tuples
        t._plan(['a'], [['b', 'sum', 's']], [('a', 'in', np.arange(3))], None)
    assert len(t._plans) == 4
    # equal-comparing values of different types are different keys
    from bqueryd_amd.engine import _freeze
    keys = [_freeze(v) for v in ([1], [1.0], [True], (1,), [np.float32(1)], [np.int64(1)], ['1'], [b'1'])]
    assert len(set(keys)) == len(keys)
    assert _freeze({'x', 'y'}) == _freeze({'y', 'x'})


def test_shard_cache_budget_counts_unions():
    """The node-level unions of a GPU's shards count against its shard cache budget: over
    budget, unions are dropped first, then the least recently used shards -- and a union built
    over an evicted shard goes with it."""
    class FakeTable:
        handle = 1

        def __init__(self, n):
            self.nrows, self.dtypes = n, OrderedDict(a=np.dtype(np.int64))

        def device_bytes(self):  # HBM held, compact copies included (bqg_table_device_bytes)
            return self.nrows * 8

    class FakeCt:
        def __init__(self, n):
            self._table, self.closed = FakeTable(n), False

        def close(self):
            self.closed = True

    class FakeUnions:
        def __init__(self):
            self.held = []  # (bytes, members)

        def bytes(self):
            return sum(b for b, _ in self.held)

        def drop_oldest(self):
            if not self.held:
                return False
            self.held.pop(0)
            return True

        def forget(self, ct):
            self.held = [(b, m) for b, m in self.held if ct not in m]

    cache = worker.ShardCache(budget_bytes=1000)
    cache.extra = FakeUnions()
    cts = {}
    for name in ('a', 'b'):
        cts[name] = FakeCt(40)  # 320 bytes each
        cache._items[(name, None)] = cts[name]
    cache.extra.held.append((300, [cts['a'], cts['b']]))
    cache._evict()
    assert cache.resident_bytes() == 940 and not cts['a'].closed
    cts['c'] = FakeCt(40)
    cache._items[('c', None)] = cts['c']
    cache._evict()  # 1260 > 1000: the union goes first (960 left)
    assert cache.extra.held == [] and not any(c.closed for c in cts.values())
    cache.extra.held.append((100, [cts['a']]))
    cts['d'] = FakeCt(10)
    cache._items[('d', None)] = cts['d']
    cache._evict()  # 1140: the union, then shard a (least recent)
    assert cache.extra.held == [] and cts['a'].closed and not cts['b'].closed
    assert cache.resident_bytes() <= 1000


@pytest.mark.parametrize('nrows', [0, 3, 100_000])
def test_ctable_tar_bytes_match_tarfile(nrows, monkeypatch):
    """The hand-written ustar blocks of bcolz_io.ctable_tar are byte-identical to what
    ``tarfile`` writes for the same members (directories first, entries sorted, depth first)."""
    import time as _time
    monkeypatch.setattr(_time, 'time', lambda: 1_700_000_000.25)
    rng = np.random.default_rng(nrows)
    cols = OrderedDict(k=rng.integers(0, 9, nrows).astype(np.int32), v=rng.normal(size=nrows))
    got = bcolz_io.ctable_tar(cols, 'result_x1')
    tree = {}
    for n in cols:
        tree.setdefault(n, {}).setdefault('data', {})
        tree[n].setdefault('meta', {})
    for rel, data in bcolz_io.ctable_files(cols):
        node = tree
        parts = rel.split('/')
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = data
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode='w') as tf:
        def add(name, node):
            info = tarfile.TarInfo(name)
            info.mtime = 1_700_000_000
            if isinstance(node, dict):
                info.type, info.mode = tarfile.DIRTYPE, 0o755
                tf.addfile(info)
                for k in sorted(node):
                    add(name + '/' + k, node[k])
            else:
                info.size, info.mode = len(node), 0o644
                tf.addfile(info, io.BytesIO(node))
        add('result_x1', tree)
    assert got == buf.getvalue()


def test_option_names_match_the_header():
    """bqueryd_amd._lib.OPTIONS (what the option tests walk) lists exactly the engine options
    include/bqgpu.h documents."""
    header = open(os.path.join(os.path.dirname(__file__), '..', 'include', 'bqgpu.h')).read()
    block = header[header.index('Engine options (ABI 6)'):header.index('int bqg_set_option')]
    names = re.findall(r'^ \*   (\w+)\s+-?\d', block, re.M)
    assert len(names) >= 20, names
    assert sorted(names) == sorted(_lib.OPTIONS), set(names) ^ set(_lib.OPTIONS)
