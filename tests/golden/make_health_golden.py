"""Known-answer vectors for the invoker health supervision (InvokerSupervision.scala).

Each case is the event sequence of a reference test (InvokerSupervisionTests.scala, "T-ISUP" below) or a timing case
derived from the akka FSM rules the reference relies on, with the expectation written BY HAND from the reference
source (not from the oracle):
  - InvokerActor starts Unhealthy; initialize() runs the _ -> Unhealthy handler: one test action + the 1-minute Tick
    timer (ISUP:305, 356-365); Ping in Offline -> Unhealthy (ISUP:308-310)
  - handleCompletionMessage (ISUP:383-410): buffer of 10, > 3 system errors -> Unhealthy, else > 3 timeouts ->
    Unresponsive, else Healthy; Healthy + Success and Offline stay; Success while Unhealthy sends a test action
  - state timeout 10 s in Unhealthy / Unresponsive / Healthy, re-armed by every processed message (Tick included)
  - handlers run in registration order (log, Unhealthy, Unresponsive): Unresponsive -> Unhealthy sets the timer in the
    Unhealthy handler and cancels it in the Unresponsive one (ISUP:339-365) -- no Tick afterwards
  - InvokerPool pads the status vector with Offline entries carrying the registering instance's userMemory
    (ISUP:180-191); messages for an invoker without an actor are dropped (ISUP:134-136)
T-ISUP's pool tests drive the child with mocked CurrentState/Transition messages; here the real actor runs, so the
state it reports right after registration is Unhealthy (its start state) where the mock sent Healthy.
Event = [kind, invoker, t_ms, userMemory bytes]; kinds: PING 0, SUCCESS 1, SYSTEM_ERROR 2, TIMEOUT 3, STATE_TIMEOUT 4
(an FSM.StateTimeout message, as T-ISUP's timeout(actor)).  Status: Healthy 0, Unhealthy 1, Unresponsive 2, Offline 3.
Run `python tests/golden/make_health_golden.py` to regenerate tests/golden/health_vectors.json.
"""
import json
import os

PING, OK, SE, TO, STO = 0, 1, 2, 3, 4
H, U, R, O = 0, 1, 2, 3
MB = 1 << 20
M = 1024 * MB  # defaultUserMemory, T-ISUP:77

CASES = []


def case(name, cite, batches, final=None):
    CASES.append({"name": name, "cite": cite, "batches": batches, "final": final or {}})


def b(events, now, status, tests):
    return {"events": events, "now": now, "status": status, "tests": tests}


# T-ISUP:99-140 -- registration pads with Offline; a repeated ping changes nothing; invoker 2 goes offline
case("pool registers on ping and tracks state changes", "T-ISUP:99-140", [
    b([[PING, 5, 0, M]], 0, [O, O, O, O, O, U], [0, 0, 0, 0, 0, 1]),
    b([[PING, 2, 0, M]], 0, [O, O, U, O, O, U], [0, 0, 1, 0, 0, 0]),
    b([[PING, 5, 0, M]], 0, [O, O, U, O, O, U], [0, 0, 0, 0, 0, 0]),
    b([[STO, 2, 0, M]], 0, [O, O, O, O, O, U], [0, 0, 0, 0, 0, 0]),
], {"mem": [M] * 6, "tick": [-1, -1, -1, -1, -1, 60000]})

# T-ISUP:246-262 and 338-353 -- Unhealthy -> Offline on a state timeout -> Unhealthy on a ping (+1 test action)
case("unhealthy, offline on timeout, unhealthy on ping", "T-ISUP:246-262, 338-353", [
    b([[PING, 0, 0, M]], 0, [U], [1]),
    b([[STO, 0, 0, M]], 0, [O], [0]),
    b([[PING, 0, 0, M]], 0, [U], [1]),
], {"tick": [60000]})


def trace(results, expect_status, expect_tests):
    return [b([[k, 0, 0, M]], 0, [s], [t]) for k, s, t in zip(results, expect_status, expect_tests)]


# T-ISUP:265-299 -- the first Success already makes it Healthy (0 errors <= 3); the 4th SystemError -> Unhealthy
# (+1 test); while Unhealthy every Success sends a test action; after 7 Successes the buffer holds 3 errors -> Healthy
case("healthy, unhealthy on system errors, healthy again", "T-ISUP:265-299",
     [b([[PING, 0, 0, M]], 0, [U], [1])]
     + trace([OK] * 10, [H] * 10, [1] + [0] * 9)
     + trace([SE] * 10, [H, H, H, U, U, U, U, U, U, U], [0, 0, 0, 1, 0, 0, 0, 0, 0, 0])
     + trace([OK] * 7, [U, U, U, U, U, U, H], [1] * 7),
     {"tick": [-1]})

# T-ISUP:302-335 -- same with timeouts: Unresponsive (+1 test); Successes while Unresponsive send no test action
case("healthy, unresponsive on timeouts, healthy again", "T-ISUP:302-335",
     [b([[PING, 0, 0, M]], 0, [U], [1])]
     + trace([OK] * 10, [H] * 10, [1] + [0] * 9)
     + trace([TO] * 10, [H, H, H, R, R, R, R, R, R, R], [0, 0, 0, 1, 0, 0, 0, 0, 0, 0])
     + trace([OK] * 7, [R, R, R, R, R, R, H], [0] * 7),
     {"tick": [-1]})

# T-ISUP:355-368 -- the Tick timer runs while Unhealthy and is cancelled on Healthy
case("test-action timer while unhealthy only", "T-ISUP:355-368", [
    b([[PING, 0, 0, M]], 0, [U], [1]),
    b([[OK, 0, 0, M]] * 7, 0, [H], [1]),
], {"tick": [-1]})

# T-ISUP:370-392 -- the status keeps the pinging instance (here: its userMemory); a restarted instance replaces it
case("status keeps the latest instance", "T-ISUP:370-392", [
    b([[PING, 0, 0, M]], 0, [U], [1]),
    b([[PING, 0, 0, 2 * M]], 0, [U], [0]),
], {"mem": [2 * M]})

# derived: the state timeout fires at last message + 10 s (due when deadline <= now)
case("state timeout at exactly 10 s", "ISUP:298, 313-331 (akka FSM stateTimeout)", [
    b([[PING, 0, 0, M]], 9999, [U], [1]),
    b([], 10000, [O], [0]),
], {"tick": [-1]})

case("every message re-arms the healthy timeout", "ISUP:326-331, 334-336", [
    b([[PING, 0, 0, M], [OK, 0, 1000, M], [PING, 0, 10999, M]], 20998, [H], [2]),
    b([], 20999, [O], [0]),
])

# derived: pings every 5 s keep an Unhealthy invoker out of Offline; Ticks at 60 s and 120 s each send a test action
case("ticks every minute while unhealthy", "ISUP:317-321, 356-361", [
    b([[PING, 0, 5000 * k, M] for k in range(26)], 125000, [U], [3]),
], {"tick": [180000]})

# derived: Unresponsive -> Unhealthy -- the Unhealthy handler sets the timer, the Unresponsive handler then cancels it
case("unresponsive to unhealthy leaves no tick timer", "ISUP:339-365 (handler order)", [
    b([[PING, 0, 0, M], [OK, 0, 0, M]] + [[TO, 0, 0, M]] * 4 + [[SE, 0, 0, M]] * 4, 0, [U], [4]),
    b([[PING, 0, 5000 * k, M] for k in range(1, 21)], 100000, [U], [0]),
], {"tick": [-1]})

# derived: a Tick re-arms the state timeout (it is a message the FSM processes)
case("a tick re-arms the state timeout", "ISUP:317-321 (Tick -> stay)", [
    b([[PING, 0, 0, M]] + [[PING, 0, 9000 * k, M] for k in range(1, 7)], 54000, [U], [1]),
    b([], 60000, [U], [1]),        # Tick at 60000 (last ping 54000 + 10 s = 64000 is later)
    b([], 69999, [U], [0]),        # re-armed by the Tick: due at 70000
    b([], 70000, [O], [0]),
], {"tick": [-1]})

# derived: padding carries the userMemory of the instance that grew the vector; later registrations replace theirs
case("padding userMemory", "ISUP:180-191", [
    b([[PING, 3, 0, 1 * M], [PING, 1, 0, 2 * M], [PING, 6, 0, 3 * M]], 0, [O, U, O, U, O, O, U], [0, 1, 0, 1, 0, 0, 1]),
], {"mem": [M, 2 * M, M, M, 3 * M, 3 * M, 3 * M]})

# derived: completions for invokers without an actor are dropped; Offline ignores completions (stays Offline)
case("messages without an actor are dropped", "ISUP:134-136, 402-404", [
    b([[OK, 4, 0, M], [SE, 0, 0, M]], 0, [], []),
    b([[PING, 0, 0, M], [OK, 7, 0, M], [STO, 0, 0, M], [SE, 0, 0, M], [SE, 0, 0, M], [SE, 0, 0, M], [SE, 0, 0, M]],
      0, [O], [1]),
    b([[PING, 0, 1, M]], 1, [U], [1]),   # the buffer kept the 4 errors: the next Success stays Unhealthy
    b([[OK, 0, 2, M]], 2, [U], [1]),
])


def main():
    # ring buffer of the system-error case: [E, E, E, S x 7] oldest first, 2 bits per result | count << 20
    for c in CASES:
        if c["name"].startswith("healthy, unhealthy"):
            c["final"]["ring"] = [(10 << 20) | sum(SE << (2 * k) for k in range(3)) | sum(OK << (2 * k) for k in range(3, 10))]
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "health_vectors.json")
    with open(out, "w") as f:
        json.dump(CASES, f, indent=1)
    print(f"wrote {len(CASES)} cases to {out}")


if __name__ == "__main__":
    main()
