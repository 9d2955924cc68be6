"""Known-answer vectors for ActivationMessage serialisation + per-invoker topic fan-out.

Expected messages are written BY HAND from the reference source, not produced by the oracle:
  - jsonFormat11(ActivationMessage.apply) member order: transid, action, revision, user, activationId,
    rootControllerIndex, blocking, content, initArgs, cause, traceContext; None options omitted (Message.scala:51-63,
    170-175); initArgs (a Set, default empty) is always written
  - TransactionId.serdes.write: ["id",start] or ["id",start,true] when extraLogging (TransactionId.scala:235-241)
  - ActivationId: 32 lowercase hex digits (ActivationId.scala:50-95); ControllerInstanceId("0") -> {"asString":"0"}
    (jsonFormat1, InstanceId.scala:40, 59)
  - spray-json CompactPrinter string escaping: \\" \\\\ \\b \\f \\n \\r \\t; other units < 0x20, DEL and non-ASCII as
    \\u + 4 lowercase hex digits (UTF-16 units: a supplementary character is a surrogate pair)
  - topics "invoker<N>", messages in publish order within a topic (CommonLoadBalancer.scala:175-198)
The `user` template below follows Identity's jsonFormat5 (subject, namespace, authkey, rights, limits) for the
ShardingContainerPoolBalancerTests identity shape; it is caller data (printed once per identity) and the vectors
check how the device assembles it.
Run `python tests/golden/make_msg_golden.py` to regenerate tests/golden/msg_vectors.json.
"""
import json
import os

UUID = "23bc46b1-71f6-4ed5-8c54-816aa4f8c502"
KEY = UUID + ":123zO3xZCLrMN6v2BKK1dXYFpXlPkccOFqm12CdAsMgRU4VrNZ9lyGVCGuMDGIwP"
USER = ('{"subject":"testspace","namespace":{"name":"testspace","uuid":"%s"},"authkey":{"api_key":"%s"},'
        '"rights":[],"limits":{}}' % (UUID, KEY))
A0 = '"action":{"path":"testspace","name":"testname","version":"0.0.1"},"revision":null,"user":' + USER
A1 = '"action":{"path":"ns/pkg","name":"act","version":"0.0.2"},"revision":"3-a1b2","user":' + USER
TEMPLATES = {"a": [A0, A1], "b": ["[]", '["a","b"]']}
RCI = '{"asString":"0"}'
AID = "0123456789abcdef0123456789abcdef"
AID2 = "fedcba98765432100123456789abcdef"
CAUSE = "00000000000000000000000000000001"


def act(invoker, tmpl, aid, tid, start, blocking=False, extra=False, content=None, cause=None, trace=None):
    return {"invoker": invoker, "tmpl": tmpl, "aid": aid, "tid": tid, "start": start, "blocking": blocking,
            "extra": extra, "content": content, "cause": cause, "trace": trace}


CASES = [
    {"name": "canonical non-blocking publish, no content", "n_topics": 1,
     "acts": [act(0, 0, AID, "sid_testing", 1700000000456)],
     "topics": [['{"transid":["sid_testing",1700000000456],' + A0 + ',"activationId":"' + AID
                 + '","rootControllerIndex":{"asString":"0"},"blocking":false,"initArgs":[]}']]},
    {"name": "blocking with content, extra logging, init args", "n_topics": 1,
     "acts": [act(0, 1, AID2, "sid_x", 1, blocking=True, extra=True, content='{"payload":"hi"}')],
     "topics": [['{"transid":["sid_x",1,true],' + A1 + ',"activationId":"' + AID2
                 + '","rootControllerIndex":{"asString":"0"},"blocking":true,"content":{"payload":"hi"},'
                   '"initArgs":["a","b"]}']]},
    {"name": "cause and traceContext after initArgs", "n_topics": 1,
     "acts": [act(0, 0, AID, "t", 0, content="{}", cause=CAUSE, trace='{"traceparent":"00-abc-01"}')],
     "topics": [['{"transid":["t",0],' + A0 + ',"activationId":"' + AID
                 + '","rootControllerIndex":{"asString":"0"},"blocking":false,"content":{},"initArgs":[],'
                   '"cause":"' + CAUSE + '","traceContext":{"traceparent":"00-abc-01"}}']]},
    {"name": "transaction id escaping (spray CompactPrinter)", "n_topics": 1,
     "acts": [act(0, 0, AID, 'a"b\\c\t\x7fé\U0001F600\x01/', 42)],
     "topics": [['{"transid":["a\\"b\\\\c\\t\\u007f\\u00e9\\ud83d\\ude00\\u0001/",42],' + A0 + ',"activationId":"'
                 + AID + '","rootControllerIndex":{"asString":"0"},"blocking":false,"initArgs":[]}']]},
    {"name": "fan-out: grouped by invoker, publish order within a topic, no message for None", "n_topics": 4,
     "acts": [act(2, 0, AID, "m0", 10), act(0, 0, AID, "m1", 11), act(2, 1, AID2, "m2", 12),
              act(-1, 0, AID, "m3", 13), act(0, 0, AID, "m4", 14)],
     "topics": [
         ['{"transid":["m1",11],' + A0 + ',"activationId":"' + AID
          + '","rootControllerIndex":{"asString":"0"},"blocking":false,"initArgs":[]}',
          '{"transid":["m4",14],' + A0 + ',"activationId":"' + AID
          + '","rootControllerIndex":{"asString":"0"},"blocking":false,"initArgs":[]}'],
         [],
         ['{"transid":["m0",10],' + A0 + ',"activationId":"' + AID
          + '","rootControllerIndex":{"asString":"0"},"blocking":false,"initArgs":[]}',
          '{"transid":["m2",12],' + A1 + ',"activationId":"' + AID2
          + '","rootControllerIndex":{"asString":"0"},"blocking":false,"initArgs":["a","b"]}'],
         []]},
]


def main():
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "msg_vectors.json")
    with open(out, "w") as f:
        json.dump({"templates": TEMPLATES, "rci": RCI, "cases": CASES}, f, indent=1, ensure_ascii=True)
    print(f"wrote {len(CASES)} cases to {out}")


if __name__ == "__main__":
    main()
