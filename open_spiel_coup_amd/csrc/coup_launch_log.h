// The per-thread launch log (coup_launch_log, include/coup_mi355x.h): each
// launch site of the step / trajectory / rollout paths notes its kernel's
// name as bench.py's roofline.kernel spells it, so the bench-size parity
// tests can assert that they ran the kernels the bench line names, and the
// bench line can report what its timed region actually enqueued.
//
// note_launch(fmt, v...): fmt holds "{}" (the next value as a decimal) and
// "{b}" (the next value as true / false); at most 5 values.  Host code only;
// a few ns per launch (formatting happens when the log is read).
#ifndef COUP_LAUNCH_LOG_H_
#define COUP_LAUNCH_LOG_H_

namespace coup {
void note_launch(const char* fmt, int v0 = 0, int v1 = 0, int v2 = 0, int v3 = 0, int v4 = 0);
}  // namespace coup

#endif  // COUP_LAUNCH_LOG_H_
