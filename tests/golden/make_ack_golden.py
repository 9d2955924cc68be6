"""Known-answer vectors for the completion-ack path (processAcknowledgement, CommonLoadBalancer.scala:205-232).

Each message is written the way the reference serialises it or as a deliberate variant, and each expectation is
derived BY HAND from the reference source (not from the oracle), citing the rule it follows:
  - canonical CompletionMessage JSON = CompletionMessage(...).serialize (ShardingContainerPoolBalancerTests.scala:574,
    AcknowledgementMessageTests.scala:74-83): jsonFormat4 field order transid, activationId, isSystemError, invoker;
    InvokerInstanceId with None options omitted; ByteSize written as "<n> MB" (Size.scala:107-114)
  - member dispatch: "invoker" + "response" -> Combined, "invoker" -> Completion, else Result (Message.scala:241-254)
  - ActivationId.parse: 32 chars of [0-9a-f] (ActivationId.scala:50-68)
  - ByteSize.fromString regex (?i)\\s?(\\d+)\\s?(GB|MB|KB|B|G|M|K)\\s? (Size.scala:119-138)
  - IntJsonFormat = BigDecimal.intValue (truncate, low 32 bits); Option members absent or null -> None
  - TransactionId.serdes read (TransactionId.scala:243-252) and equality with invokerHealth (id, start, extraLogging)
The vectors are data: run `python tests/golden/make_ack_golden.py` to regenerate tests/golden/ack_vectors.json.
Kinds: FAIL 0, JVM 1 (response member, deserialised by the JVM), UNSUPPORTED 2 (device parser limits), COMPLETION 3.
"""
import json
import os

H = 1700000000123  # TransactionId.invokerHealth start (ms) of the controller under test
AID = "0123456789abcdef0123456789abcdef"
TID = '["sid_testing",1700000000456]'
INV = '{"instance":%s,"userMemory":"1024 MB"}'


def completion(aid=f'"{AID}"', sys="false", inv=INV % "0", tid=TID):
    return '{"transid":%s,"activationId":%s,"isSystemError":%s,"invoker":%s}' % (tid, aid, sys, inv)


V = []


def add(name, msg, kind, instance=None, syserr=0, health=0, aid=AID):
    e = {"name": name, "msg": msg, "kind": kind}
    if kind == 3:
        e.update(instance=instance, syserr=syserr, health=health, aid=aid)
    V.append(e)


add("canonical completion (T-SCPB:574)", completion(), 3, 0)
add("system error true", completion(sys="true"), 3, 0, syserr=1)
add("system error null -> None -> false", completion(sys="null"), 3, 0)
add("system error absent", '{"transid":%s,"activationId":"%s","invoker":%s}' % (TID, AID, INV % "7"), 3, 7)
add("system error as string", completion(sys='"false"'), 0)
add("instance 3.7 -> intValue 3", completion(inv=INV % "3.7"), 3, 3)
add("instance 2^32+3 -> low 32 bits", completion(inv=INV % "4294967299"), 3, 3)
add("instance -1", completion(inv=INV % "-1"), 3, -1)
add("instance 1e2", completion(inv=INV % "1e2"), 3, 100)
add("instance 12.5E1", completion(inv=INV % "12.5E1"), 3, 125)
add("instance as string", completion(inv=INV % '"0"'), 0)
add("invoker without userMemory", completion(inv='{"instance":0}'), 0)
add("userMemory lower case, spaces", completion(inv='{"instance":1,"userMemory":" 2048mb "}'), 3, 1)
add("userMemory G", completion(inv='{"instance":1,"userMemory":"4G"}'), 3, 1)
add("userMemory two spaces", completion(inv='{"instance":1,"userMemory":"1024  MB"}'), 0)
add("userMemory unit XB", completion(inv='{"instance":1,"userMemory":"1024 XB"}'), 0)
add("userMemory Long overflow", completion(inv='{"instance":1,"userMemory":"99999999999999999999 MB"}'), 0)
add("userMemory escaped digit", completion(inv='{"instance":1,"userMemory":"\\u0031 MB"}'), 3, 1)
add("uniqueName and displayedName", completion(inv='{"instance":2,"uniqueName":"u","displayedName":null,'
                                                   '"userMemory":"1 B"}'), 3, 2)
add("uniqueName number", completion(inv='{"instance":2,"uniqueName":5,"userMemory":"1 B"}'), 0)
add("invoker not an object", completion(inv="[0]"), 0)
add("activation id 31 chars", completion(aid='"%s"' % AID[:31]), 0)
add("activation id upper case hex", completion(aid='"%s"' % AID.upper()), 0)
add("activation id escaped a", completion(aid='"0123456789\\u0061bcdef0123456789abcdef"'), 3, 0)
add("activation id as number", completion(aid="12345678901234567890123456789012"), 2)
add("activation id null", completion(aid="null"), 0)
add("activation id non-ASCII digit", completion(aid='"0123456789abcdef0123456789abcde\\u0663"'), 2)
add("missing transid", '{"activationId":"%s","invoker":%s}' % (AID, INV % "0"), 0)
add("transid of another shape is fine", completion(tid='"x"'), 3, 0)
add("missing activationId", '{"transid":%s,"invoker":%s}' % (TID, INV % "0"), 0)
add("result message, Left (AcknowledgementMessageTests:57-64)", '{"transid":%s,"response":"%s"}' % (TID, AID), 1)
add("combined message", '{"transid":%s,"response":"%s","isSystemError":false,"invoker":%s}' % (TID, AID, INV % "0"),
    1)
add("result member without invoker and response", '{"transid":%s,"activationId":"%s"}' % (TID, AID), 0)
add("escaped member name", completion().replace('"invoker"', '"inv\\u006fker"'), 3, 0)
add("duplicate invoker: last wins", completion()[:-1] + ',"invoker":' + INV % "9" + "}", 3, 9)
add("whitespace everywhere", " \n" + completion().replace(",", " ,\t").replace(":", " : ") + "\r\n ", 3, 0)
add("trailing garbage", completion() + "x", 0)
add("top-level array", "[" + completion() + "]", 0)
add("empty", "", 0)
add("truncated", completion()[:-1], 0)
add("raw control character in a string", completion(inv='{"instance":0,"userMemory":"1024\\tMB","x":"a\tb"}'), 0)
add("invalid escape", completion(inv='{"instance":0,"userMemory":"1024 MB","x":"\\q"}'), 0)
add("leading zero number", completion(inv=INV % "01"), 0)
add("bad literal", completion(sys="fals"), 0)
add("health ack", completion(tid='["sid_invokerHealth",%d]' % H), 3, 0, health=1)
add("health ack, extraLogging false", completion(tid='["sid_invokerHealth",%d,false]' % H), 3, 0, health=1)
add("health id, extraLogging true", completion(tid='["sid_invokerHealth",%d,true]' % H), 3, 0, health=0)
add("health id, other start", completion(tid='["sid_invokerHealth",%d]' % (H + 1)), 3, 0, health=0)
add("health id, start as 1.700000000123e12", completion(tid='["sid_invokerHealth",1.700000000123e12]'), 3, 0,
    health=1)
add("deep nesting (65 levels) in another member", completion()[:-1] + ',"x":' + "[" * 64 + "]" * 64 + "}", 2)
add("nesting of 64 levels is fine", completion()[:-1] + ',"x":' + "[" * 63 + "]" * 63 + "}", 3, 0)
add("exponent of 10 digits", completion()[:-1] + ',"x":1e1234567890}', 2)
add("U+FFFF in a string", completion()[:-1] + ',"x":"￿"}', 2)
add("non-ASCII in other strings", completion()[:-1] + ',"x":"café"}', 3, 0)

if __name__ == "__main__":
    out = {"health_start_ms": H, "vectors": V}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ack_vectors.json"), "w",
              encoding="utf-8") as f:
        json.dump(out, f, indent=1, ensure_ascii=False)
    print(len(V), "vectors")
