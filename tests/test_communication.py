"""In-memory / collective protocol behaviour (reference: test/communication/communication_test.py)."""

import time

import pytest

from myfyp_amd.communication.commands.command import Command
from myfyp_amd.communication.protocols.exceptions import ProtocolNotStartedError
from myfyp_amd.communication.protocols.gossiper import Gossiper
from myfyp_amd.communication.protocols.memory.memory_communication_protocol import InMemoryCommunicationProtocol, ServerRegistry
from myfyp_amd.settings import Settings
from myfyp_amd.utils.utils import wait_convergence


class MockCommand(Command):
    def __init__(self):
        self.calls = []

    @staticmethod
    def get_name():
        return "mock_command"

    def execute(self, source, round, *args, **kwargs):
        self.calls.append((source, round, args))


@pytest.fixture
def protocols():
    made = []

    def make(n):
        for i in range(n):
            p = InMemoryCommunicationProtocol(f"comm-{len(made)}-{time.time_ns()}")
            p.start()
            made.append(p)
        return made[-n:]

    yield make
    for p in made:
        try:
            p.stop()
        except Exception:
            pass


def test_not_started_errors():
    p = InMemoryCommunicationProtocol("lonely")
    with pytest.raises(ProtocolNotStartedError):
        p.connect("x")
    with pytest.raises(ProtocolNotStartedError):
        p.broadcast(p.build_msg("beat", ["1"]))


def test_invalid_connect(protocols):
    (p,) = protocols(1)
    assert p.connect("does-not-exist") is False
    assert p.connect(p.get_address()) is False  # cannot add itself


def test_command_delivery_and_unknown(protocols):
    a, b = protocols(2)
    cmd = MockCommand()
    b.add_command(cmd)
    assert a.connect(b.get_address())
    a.send(b.get_address(), a.build_msg("mock_command", ["x", "y"], round=3))
    assert cmd.calls == [(a.get_address(), 3, ("x", "y"))]
    res = b.handle_message(a.build_msg("nope"))
    assert "error" in res
    # duplicate hash is dropped
    msg = a.build_msg("mock_command", ["z"])
    b.handle_message(msg)
    b.handle_message(msg)
    assert len(cmd.calls) == 2


def test_heartbeat_membership_relay_and_eviction(protocols):
    ps = protocols(5)
    # line topology: full membership must converge through TTL-relayed heartbeats
    for i in range(4):
        ps[i].connect(ps[i + 1].get_address())
    wait_convergence(ps, 4, only_direct=False, wait=10)
    assert len(ps[2].get_neighbors(only_direct=True)) == 2
    # abrupt crash of the middle node (no disconnect messages): heartbeat timeout evicts it
    dead = ps[2]
    dead._heartbeater.stop()
    dead._gossiper.stop()
    ServerRegistry.unregister(dead.get_address())
    dead._started = False
    t0 = time.time()
    while time.time() - t0 < 3 * Settings.HEARTBEAT_TIMEOUT + 2 and any(dead.get_address() in p.get_neighbors() for p in ps if p is not dead):
        time.sleep(0.1)
    assert all(dead.get_address() not in p.get_neighbors() for p in ps if p is not dead)
    assert time.time() - t0 >= Settings.HEARTBEAT_TIMEOUT * 0.5  # detected by timeout, not by a message


def test_disconnect(protocols):
    a, b = protocols(2)
    a.connect(b.get_address())
    assert b.get_address() in a.get_neighbors(only_direct=True)
    a.disconnect(b.get_address())
    assert b.get_address() not in a.get_neighbors(only_direct=True)
    assert a.get_address() not in b.get_neighbors(only_direct=True)


def test_gossiper_dedup_ring_and_exit():
    g = Gossiper("g", client=None)
    assert g.check_and_set_processed(1) and not g.check_and_set_processed(1)
    for i in range(Settings.AMOUNT_LAST_MESSAGES_SAVED + 5):
        g.check_and_set_processed(1000 + i)
    assert g.check_and_set_processed(1)  # evicted from the ring

    class C:
        sent = []

        def send(self, nei, msg, create_connection=False):
            self.sent.append(nei)

    g._client = C()
    calls = {"n": 0}

    def candidates():
        calls["n"] += 1
        return ["x"]

    t0 = time.time()
    g.gossip_weights(lambda: False, candidates, lambda: "same", lambda n: {"m": 1}, period=0.0, create_connection=False)
    assert calls["n"] == Settings.GOSSIP_EXIT_ON_X_EQUAL_ROUNDS and time.time() - t0 < 2


def test_registry_stop_only_unregisters_self(protocols):
    a, b = protocols(2)
    a.stop()
    assert ServerRegistry.get(a.get_address()) is None
    assert ServerRegistry.get(b.get_address()) is b
