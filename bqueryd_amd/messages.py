"""bqueryd wire messages, byte-compatible with the Python-2 reference (bqueryd/messages.py).

``Message`` is a JSON dict with ``payload``, ``version``, ``msg_type`` and ``created``
(messages.py:27-37).  Binary fields are ``cPickle.dumps(v).encode('base64')`` in the
reference (messages.py:50-56): pickle protocol 0 text encoded as MIME base64 (76-column lines,
trailing newline).  Python 3 reads them with ``encoding='latin1'`` (py2 ``str`` -> ``str``)
and writes protocol 2, which Python 2's cPickle loads.
"""
from __future__ import annotations

import base64
import json
import pickle
import time


def msg_factory(msg):
    """messages.py:6-20."""
    if isinstance(msg, (bytes, bytearray)):
        msg = msg.decode('utf-8')
    if isinstance(msg, str):
        try:
            msg = json.loads(msg)
        except ValueError:
            msg = None
    if not msg:
        return Message()
    mapping = {'calc': CalcMessage, 'rpc': RPCMessage, 'error': ErrorMessage,
               'worker_register': WorkerRegisterMessage, 'busy': BusyMessage, 'done': DoneMessage,
               'ticketdone': TicketDoneMessage, 'stop': StopMessage, None: Message}
    return mapping.get(msg.get('msg_type'), Message)(msg)


class MalformedMessage(Exception):
    pass


def encode_binary(value):
    return base64.encodebytes(pickle.dumps(value, protocol=2)).decode('ascii')


def decode_binary(buf):
    if isinstance(buf, str):
        buf = buf.encode('latin1')
    return pickle.loads(base64.decodebytes(buf), encoding='latin1')


class Message(dict):
    msg_type = None

    def __init__(self, datadict=None):
        if datadict is None:
            datadict = {}
        super().__init__()
        self.update(datadict)
        self['payload'] = datadict.get('payload')
        self['version'] = datadict.get('version', 1)
        self['msg_type'] = self.msg_type
        self['created'] = time.time()

    def copy(self):
        return msg_factory(dict(self))

    def isa(self, payload_or_instance):
        if self.msg_type == getattr(payload_or_instance, 'msg_type', '_'):
            return True
        return self.get('payload') == payload_or_instance

    def add_as_binary(self, key, value):
        self[key] = encode_binary(value)

    def get_from_binary(self, key, default=None):
        buf = self.get(key)
        if not buf:
            return default
        return decode_binary(buf)

    def to_json(self):
        return json.dumps({k: v for k, v in self.items() if k != 'data'})

    def set_args_kwargs(self, args, kwargs):
        self.add_as_binary('params', {'args': args, 'kwargs': kwargs})

    def get_args_kwargs(self):
        params = self.get_from_binary('params', {})
        return params.get('args', []), params.get('kwargs', {})


class WorkerRegisterMessage(Message):
    msg_type = 'worker_register'


class CalcMessage(Message):
    msg_type = 'calc'


class RPCMessage(Message):
    msg_type = 'rpc'


class ErrorMessage(Message):
    msg_type = 'error'


class BusyMessage(Message):
    msg_type = 'busy'


class DoneMessage(Message):
    msg_type = 'done'


class StopMessage(Message):
    msg_type = 'stop'


class TicketDoneMessage(Message):
    msg_type = 'ticketdone'
