"""Simulator <-> learner IPC: RL/simulator.py:40-200 and the
serialisation of utils/serialize.py, without ZMQ (not installed here).

Protocol (unchanged from the reference):
  * each simulator process PUSHes `(identity, state, reward, isOver, ts, isAlive)` on the c2s
    pipe (simulator.py:95-98) and then waits on its DEALER end of the s2c pipe for
    `(action, ts, isAlive)` (:100); on isAlive == False it answers
    `(identity, 0, 0, 0, 0, False)` and exits (:101-106);
  * the master PULLs the c2s messages, keeps each client's memory (:160-185) and ROUTEs the
    reply to the identity that asked.
Messages are msgpack with numpy arrays as msgpack_numpy encodes them (serialize.py:7-20).

Transport: `ipc://<path>` addresses are Unix-domain stream sockets with 4-byte length-prefixed
frames; the s2c connection announces its identity first (the ROUTER/DEALER identity
handshake).  Kernel socket buffers provide the back-pressure ZMQ's high-water marks gave.

Masters:
  * `SimulatorMaster` — the reference's per-message master thread with the abstract
    `_on_state` / `_on_episode_over` / `_on_datapoint` hooks and host `_parse_memory`
    (train.py:394-437), for players of any kind.
  * `BatchedSimulatorMaster` (ba3c_amd.simulator_gpu) — the MI355X design: one round collects a
    state from every simulator, then ONE predictor forward + sampling for all of them and the
    per-client memories / n-step returns in HBM (ba3c_amd.rollout).
"""
import multiprocessing as mp
import os
import selectors
import socket
import struct
import threading
import time
from collections import defaultdict

import msgpack
import numpy as np

GAMMA = 0.99              # train.py:94
LOCAL_TIME_MAX = 5        # train.py:102


# ---- serialisation (utils/serialize.py + msgpack_numpy's ndarray encoding) ---------------
def _enc(obj):
    if isinstance(obj, np.ndarray):
        if obj.dtype.kind in "OV":
            raise TypeError("object / void arrays are not serialisable")
        a = np.ascontiguousarray(obj)
        return {b"nd": True, b"type": a.dtype.str, b"kind": b"", b"shape": list(a.shape),
                b"data": a.tobytes()}
    if isinstance(obj, np.generic):
        return {b"nd": False, b"type": obj.dtype.str, b"data": obj.tobytes()}
    raise TypeError("cannot serialise %r" % type(obj))


def _dec(d):
    if b"nd" in d:
        dt = np.dtype(d[b"type"])
        if d[b"nd"]:
            return np.frombuffer(d[b"data"], dtype=dt).reshape(d[b"shape"])
        return np.frombuffer(d[b"data"], dtype=dt)[0]
    return d


def dumps(obj):
    """serialize.py:13-15."""
    return msgpack.packb(obj, use_bin_type=True, default=_enc)


def loads(buf):
    """serialize.py:17-19 (tuples come back as lists, as with msgpack)."""
    return msgpack.unpackb(buf, raw=False, object_hook=_dec, strict_map_key=False)


# ---- transport -------------------------------------------------------------------------
def _path(addr):
    if not addr.startswith("ipc://"):
        raise ValueError("only ipc:// pipes are supported: %r" % addr)
    return addr[len("ipc://"):]


def _send_frame(sock, payload):
    sock.sendall(struct.pack("<I", len(payload)) + payload)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("peer closed")
        buf += chunk
    return bytes(buf)


def _recv_frame(sock):
    (n,) = struct.unpack("<I", _recv_exact(sock, 4))
    return _recv_exact(sock, n)


def _connect(addr, timeout=60.0):
    path = _path(addr)
    t0 = time.time()
    while True:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        try:
            s.connect(path)
            return s
        except (FileNotFoundError, ConnectionRefusedError):
            s.close()
            if time.time() - t0 > timeout:
                raise
            time.sleep(0.01)


def _listen(addr):
    path = _path(addr)
    if os.path.exists(path):
        os.unlink(path)
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.bind(path)
    s.listen(1024)
    return s


class PullSocket(object):
    """Master end of c2s: frames from every connected PUSH client, in arrival order."""

    def __init__(self, addr):
        self.lsock = _listen(addr)
        self.lsock.setblocking(False)
        self.sel = selectors.DefaultSelector()
        self.sel.register(self.lsock, selectors.EVENT_READ, None)
        self.bufs = {}
        self.ready = []

    def _pump(self, timeout):
        for key, _ in self.sel.select(timeout):
            if key.data is None:
                conn, _ = self.lsock.accept()
                conn.setblocking(False)
                self.bufs[conn] = bytearray()
                self.sel.register(conn, selectors.EVENT_READ, conn)
                continue
            conn = key.data
            try:
                chunk = conn.recv(1 << 20)
            except BlockingIOError:
                continue
            if not chunk:
                self.sel.unregister(conn)
                conn.close()
                del self.bufs[conn]
                continue
            buf = self.bufs[conn]
            buf += chunk
            while len(buf) >= 4:
                (n,) = struct.unpack_from("<I", buf)
                if len(buf) < 4 + n:
                    break
                self.ready.append(bytes(buf[4:4 + n]))
                del buf[:4 + n]

    def recv(self, timeout=None):
        """Next frame; None if `timeout` seconds pass without one."""
        t0 = time.time()
        while not self.ready:
            left = None if timeout is None else max(0.0, timeout - (time.time() - t0))
            if left == 0.0 and timeout is not None:
                return None
            self._pump(left if left is not None else 1.0)
        return self.ready.pop(0)

    def close(self):
        for conn in list(self.bufs):
            conn.close()
        self.sel.close()
        self.lsock.close()


class RouterSocket(object):
    """Master end of s2c: `send_multipart([identity, payload])` to the DEALER that announced
    `identity`; connections are accepted by a background thread."""

    def __init__(self, addr):
        self.lsock = _listen(addr)
        self.conns = {}
        self.cv = threading.Condition()
        self._closed = False
        self._t = threading.Thread(target=self._accept, daemon=True)
        self._t.start()

    def _accept(self):
        while not self._closed:
            try:
                conn, _ = self.lsock.accept()
            except OSError:
                return
            ident = _recv_frame(conn)
            with self.cv:
                self.conns[ident] = conn
                self.cv.notify_all()

    def send_multipart(self, msg, timeout=60.0):
        ident, payload = msg
        with self.cv:
            if not self.cv.wait_for(lambda: ident in self.conns, timeout):
                raise TimeoutError("no s2c connection from %r" % ident)
            conn = self.conns[ident]
        _send_frame(conn, payload)

    def close(self):
        self._closed = True
        try:
            self.lsock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.lsock.close()
        for c in self.conns.values():
            c.close()


# ---- simulator processes ---------------------------------------------------------------
class TransitionExperience(object):
    """simulator.py:40-48."""

    def __init__(self, state, action, reward, **kwargs):
        self.state = state
        self.action = action
        self.reward = reward
        for k, v in kwargs.items():
            setattr(self, k, v)


class SimulatorProcessStateExchange(mp.Process):
    """simulator.py:50-109: builds its player, then loops state -> action -> step."""

    def __init__(self, idx, pipe_c2s, pipe_s2c):
        super(SimulatorProcessStateExchange, self).__init__()
        self.idx = int(idx)
        self.identity = u"simulator-{}".format(self.idx).encode("utf-8")
        self.c2s = pipe_c2s
        self.s2c = pipe_s2c
        self.daemon = True

    def _build_player(self):
        raise NotImplementedError()

    def run(self):
        player = self._build_player()
        c2s = _connect(self.c2s)
        s2c = _connect(self.s2c)
        _send_frame(s2c, self.identity)
        state = player.current_state()
        reward, is_over, ts = 0, False, 0
        try:
            while True:
                _send_frame(c2s, dumps((self.identity, state, reward, is_over, ts, True)))
                action, ts, alive = loads(_recv_frame(s2c))
                if not alive:
                    _send_frame(c2s, dumps((self.identity, 0, 0, 0, 0, False)))
                    break
                reward, is_over = player.action(action)
                state = player.current_state()
        except ConnectionError:
            pass
        finally:
            c2s.close()
            s2c.close()


SimulatorProcess = SimulatorProcessStateExchange     # simulator.py:111-112


class SyntheticSimulatorWorker(SimulatorProcess):
    """MySimulatorWorker (train.py:134-136) over the synthetic game."""

    def __init__(self, idx, pipe_c2s, pipe_s2c, num_actions=4, seed=0):
        super(SyntheticSimulatorWorker, self).__init__(idx, pipe_c2s, pipe_s2c)
        self.num_actions = num_actions
        self.seed = seed

    def _build_player(self):
        from .envs import get_player
        return get_player(self.idx, self.num_actions, self.seed + self.idx, train=True)


def client_index(identity):
    """b'simulator-7' -> 7."""
    return int(identity.decode("utf-8").rsplit("-", 1)[1])


# ---- the reference's per-message master -----------------------------------------------
class SimulatorMaster(threading.Thread):
    """simulator.py:114-200 + MySimulatorMaster's memory callbacks (train.py:394-437).

    Subclasses implement `_on_state(state, (ident, ts))`, which must eventually call
    `send(ident, action, global_step)` and append a TransitionExperience(state, action, None,
    value=..., ts=ts) to `self.clients[ident].memory`.  Datapoints
    `[state, action, R, ts, init_R, isOver]` go to `self.queue` (a list, or anything with
    `put`)."""

    class ClientState(object):
        def __init__(self):
            self.memory = []

    def __init__(self, pipe_c2s, pipe_s2c, simulator_procs, local_time_max=LOCAL_TIME_MAX,
                 gamma=GAMMA):
        super(SimulatorMaster, self).__init__()
        self.daemon = True
        self.c2s_socket = PullSocket(pipe_c2s)
        self.s2c_socket = RouterSocket(pipe_s2c)
        self.simulator_procs = simulator_procs
        self.killed_threads = 0
        self.local_time_max = local_time_max
        self.gamma = gamma
        self.clients = defaultdict(self.ClientState)
        self.queue = []
        self.is_done = False
        self._stop_req = threading.Event()
        self.messages = 0

    def send(self, ident, action, global_step=0, alive=True):
        self.s2c_socket.send_multipart([ident, dumps((action, global_step, alive))])

    def stop(self):
        """Ask every client to exit: the next reply to each is (0, 0, False)."""
        self._stop_req.set()

    def handle(self, msg):
        """One c2s message (simulator.py:163-185).  Returns False when the master is done."""
        ident, state, reward, is_over, ts, alive = msg
        if not alive:
            self.killed_threads += 1
            if self.killed_threads == self.simulator_procs:
                self.is_done = True
                return False
            return True
        if self._stop_req.is_set():
            self.send(ident, 0, 0, alive=False)
            return True
        client = self.clients[ident]
        if len(client.memory) > 0:
            client.memory[-1].reward = reward
            if is_over:
                self._on_episode_over((ident, ts))
            else:
                self._on_datapoint((ident, ts))
        self._on_state(state, (ident, ts))
        return True

    def run(self):
        while True:
            buf = self.c2s_socket.recv(timeout=1.0)
            if buf is None:
                continue
            self.messages += 1
            if not self.handle(loads(buf)):
                break

    def close(self):
        self.c2s_socket.close()
        self.s2c_socket.close()

    def _on_state(self, state, ident):
        raise NotImplementedError()

    def _on_episode_over(self, ident):
        ident, ts = ident
        self._parse_memory(0, ident, True, ts)

    def _on_datapoint(self, ident):
        ident, ts = ident
        client = self.clients[ident]
        if len(client.memory) == self.local_time_max + 1:
            self._parse_memory(client.memory[-1].value, ident, False, ts)

    def _put(self, dp):
        if hasattr(self.queue, "put"):
            self.queue.put(dp)
        else:
            self.queue.append(dp)

    def _parse_memory(self, init_r, ident, is_over, ts):
        """train.py:418-437: n-step returns over the reversed memory, R = clip(r, -1, 1) +
        GAMMA * R, bootstrapped from init_r."""
        client = self.clients[ident]
        mem = client.memory
        last = None
        if not is_over:
            last = mem[-1]
            mem = mem[:-1]
        mem = mem[::-1]
        R = float(init_r)
        for k in mem:
            R = np.clip(k.reward, -1, 1) + self.gamma * R
            self._put([k.state, k.action, R, getattr(k, "ts", ts), init_r, is_over])
        client.memory = [last] if not is_over else []


class FunctionSimulatorMaster(SimulatorMaster):
    """A per-message master whose policy is `policy(state) -> (distrib, value)`, with the
    action drawn by `np.random.choice(len(distrib), p=distrib)` from `rs` (train.py:374-390)."""

    def __init__(self, pipe_c2s, pipe_s2c, simulator_procs, policy, rs=None, **kw):
        super(FunctionSimulatorMaster, self).__init__(pipe_c2s, pipe_s2c, simulator_procs, **kw)
        self.policy = policy
        self.rs = rs if rs is not None else np.random.RandomState(0)
        self.global_step = 0

    def _on_state(self, state, ident):
        ident, ts = ident
        distrib, value = self.policy(state)
        assert np.all(np.isfinite(distrib)), distrib
        action = int(self.rs.choice(len(distrib), p=distrib))
        self.clients[ident].memory.append(TransitionExperience(state, action, None, value=value, ts=ts))
        self.send(ident, action, self.global_step)


def start_simulators(worker_cls, n, pipe_c2s, pipe_s2c, threads=False, **kw):
    """Start `n` simulators (train.py:520-523).  As processes (the reference's layout) they
    are forked, so start them BEFORE the learner initialises the GPU, as the reference starts
    them before its session; `threads=True` runs the same `run()` loops as threads of this
    process instead (same sockets, same protocol), for a process that already holds the GPU."""
    workers = [worker_cls(i, pipe_c2s, pipe_s2c, **kw) for i in range(n)]
    if threads:
        ts = [threading.Thread(target=w.run, daemon=True) for w in workers]
        for t in ts:
            t.start()
        return ts
    for w in workers:
        w.start()
    return workers
