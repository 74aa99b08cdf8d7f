"""NodeState.clear (a network-wide stop) must wake every thread blocked on the state's primitives,
including a StartLearningStage still waiting for the initial model (parity:
/root/reference/p2pfl/node_state.py clear, /root/reference/p2pfl/stages/base_node/start_learning_stage.py)."""

import threading
import time

from myfyp_amd.node_state import NodeState


def test_clear_wakes_a_start_stage_waiting_for_the_initial_model():
    st = NodeState("state-a")
    st.set_experiment("exp", 3)
    old = st.model_initialized_lock
    woke = threading.Event()
    seen = []

    def waiter():  # what StartLearningStage does: acquire, then check the round
        old.acquire()
        seen.append(st.round)
        woke.set()

    t = threading.Thread(target=waiter, daemon=True)
    t.start()
    time.sleep(0.05)
    assert not woke.is_set()
    st.clear()  # the stop arrives before the initial model
    assert woke.wait(2.0), "a stage waiting for the initial model stayed blocked after clear()"
    assert seen == [None]  # it sees the cleared round and ends the workflow
    # the fresh state waits for a new initial model again
    assert st.model_initialized_lock is not old and st.model_initialized_lock.locked()
    t.join(1.0)


def test_clear_without_a_waiter_leaves_a_locked_fresh_lock():
    st = NodeState("state-b")
    st.clear()
    st.clear()
    assert st.round is None and st.model_initialized_lock.locked()
