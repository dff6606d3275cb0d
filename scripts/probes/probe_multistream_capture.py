"""Which multi-stream hipGraph capture patterns does this torch/HIP stack accept?  Each
case runs in a child process (a crash in one does not hide the others); prints one line
per case."""
import subprocess
import sys

CASES = {
    "fork_join": """
y = None
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev)
with torch.cuda.stream(s1):
    y = x * 2
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
z = y + 1
g.capture_end()
""",
    "fork_join_set_stream": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev)
torch.cuda.set_stream(s1)
y = x * 2
torch.cuda.set_stream(main)
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
z = y + 1
g.capture_end()
""",
    "record_stream": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev)
w = x * 3
w.record_stream(s1)
with torch.cuda.stream(s1):
    y = w * 2
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
z = y + 1
g.capture_end()
""",
    "unwaited_event": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev)
with torch.cuda.stream(s1):
    y = x * 2
    e3 = torch.cuda.Event(); e3.record(s1)
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
z = y + 1
g.capture_end()
""",
    "free_on_lane": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev)
with torch.cuda.stream(s1):
    t = x * 2
    y = t + 1
    del t
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
z = y + 1
g.capture_end()
""",
    "two_lanes_cross": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev); s2.wait_event(ev)
with torch.cuda.stream(s1):
    a = x * 2
    ea = torch.cuda.Event(); ea.record(s1)
with torch.cuda.stream(s2):
    b = x * 3
    s2.wait_event(ea)
    c = a + b
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
ev3 = torch.cuda.Event(); ev3.record(s2); main.wait_event(ev3)
z = c + 1
g.capture_end()
""",
    "empty_lane": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev)
z = x * 2
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
z = z + 1
g.capture_end()
""",
    "lane_waits_only": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev); s2.wait_event(ev)
with torch.cuda.stream(s1):
    a = x * 2
    ea = torch.cuda.Event(); ea.record(s1)
s2.wait_event(ea)
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
ev3 = torch.cuda.Event(); ev3.record(s2); main.wait_event(ev3)
z = a + 1
g.capture_end()
""",
    "double_wait_same_event": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev)
with torch.cuda.stream(s1):
    a = x * 2
    ea = torch.cuda.Event(); ea.record(s1)
main.wait_event(ea)
main.wait_event(ea)
b = a + 1
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
z = b + 1
g.capture_end()
""",
    "join_twice": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev)
with torch.cuda.stream(s1):
    a = x * 2
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
ev4 = torch.cuda.Event(); ev4.record(s1); main.wait_event(ev4)
z = a + 1
g.capture_end()
""",
    "three_side_lanes": """
g.capture_begin(pool=pool)
s3 = torch.cuda.Stream()
ev = torch.cuda.Event(); ev.record(main)
outs = []
for s in (s1, s2, s3):
    s.wait_event(ev)
    with torch.cuda.stream(s):
        outs.append(x * 2)
for s in (s1, s2, s3):
    e = torch.cuda.Event(); e.record(s); main.wait_event(e)
z = outs[0] + outs[1] + outs[2]
g.capture_end()
""",
    "events_destroyed_before_end": """
g.capture_begin(pool=pool)
def fork(s):
    ev = torch.cuda.Event(); ev.record(main); s.wait_event(ev)
def join(s):
    ev = torch.cuda.Event(); ev.record(s); main.wait_event(ev)
fork(s1); fork(s2)
with torch.cuda.stream(s1):
    a = x * 2
with torch.cuda.stream(s2):
    b = x * 3
join(s1); join(s2)
import gc; gc.collect()
z = a + b
g.capture_end()
""",
    "record_stream_then_free": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev)
w = x * 3
w.record_stream(s1)
with torch.cuda.stream(s1):
    y = w * 2
del w
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
z = y + 1
g.capture_end()
""",
    "lane_alloc_free_on_main": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev)
with torch.cuda.stream(s1):
    w = x * 3
e1 = torch.cuda.Event(); e1.record(s1); main.wait_event(e1)
w.record_stream(main)
y = w * 2
del w
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
z = y + 1
g.capture_end()
""",
    "record_stream_outside_tensor": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev)
x.record_stream(s1)
with torch.cuda.stream(s1):
    y = x * 2
ev2 = torch.cuda.Event(); ev2.record(s1); main.wait_event(ev2)
z = y + 1
g.capture_end()
""",
    "lane_set_stream_raw_launch": """
g.capture_begin(pool=pool)
ev = torch.cuda.Event(); ev.record(main); s1.wait_event(ev)
torch.cuda.set_stream(s1)
y = torch.empty_like(x); y.copy_(x)
torch.cuda.set_stream(main)
e1 = torch.cuda.Event(); e1.record(s1); main.wait_event(e1)
z = y + 1
g.capture_end()
""",
}

PRE = """
import torch
x = torch.ones(1024, device="cuda")
main = torch.cuda.Stream(); s1 = torch.cuda.Stream(); s2 = torch.cuda.Stream()
pool = torch.cuda.graph_pool_handle()
torch.cuda.synchronize()
with torch.cuda.stream(main):
    g = torch.cuda.CUDAGraph()
"""
POST = """
g.replay(); torch.cuda.synchronize(); print("ok", float(z.sum()))
"""


def main():
    for name, body in CASES.items():
        body = "\n".join("    " + ln for ln in body.strip().splitlines())
        code = PRE + body + "\n" + POST
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                           timeout=120)
        tail = (r.stdout.strip().splitlines() or [""])[-1]
        err = (r.stderr.strip().splitlines() or [""])[-1]
        print(f"{name}: rc={r.returncode} {tail} {err[:160] if r.returncode else ''}",
              flush=True)


if __name__ == "__main__":
    main()
