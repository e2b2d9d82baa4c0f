// hipps runtime — shared-memory control plane for the asynchronous parameter server.
//
// MPI gives the reference an any-source receive (README.md:65-70 `recv(MPI.ANY_SOURCE)`); RCCL
// has none.  On one node hipps replaces it with a POSIX shared-memory control block: each rank
// owns a cache-line-padded record of sequence words (gradient pushed / consumed, version used,
// stop), and the PS owns the published-parameter version words.  Data never goes through here
// (it moves device-to-device into IPC mailboxes, see ipc.cpp); only 8-byte doorbells do.
//
//   worker: copy grad -> PS mailbox slot (comm stream) ; then doorbell -> push_seq = s
//   PS:     wait_any(push_seq > seen) ; accumulate slot ; doorbell -> ack_seq = s
//   PS:     after M grads: update + publish into a free pub buffer b ; doorbell -> buf_ver[b], pub_ver
//   worker: irequest_params(): pub_ver newer? reading = v ; copy pub[b] (one-sided pull) ;
//           doorbell -> reading = -1   (the PS never rewrites a buffer somebody is reading)
//
// Doorbells are stream-ordered: a one-wavefront kernel (doorbell.hip) stores the words with a
// system-scope release into this block, which every process registers with hipHostRegister.
// Without a HIP device (CPU runs) or if registration fails they fall back to
// hipLaunchHostFunc callbacks.  Either way a doorbell never runs ahead of the bytes it announces.
#include "runtime/control.h"

namespace hipps {
namespace rt {

void bind_control(py::module& m) {
  py::class_<ControlBlock>(m, "ControlBlock")
      .def(py::init<const std::string&, int, bool>(), py::arg("name"), py::arg("world"), py::arg("create"))
      .def("unlink", &ControlBlock::unlink)
      .def("load", &ControlBlock::load)
      .def("store", &ControlBlock::store)
      .def("fetch_add", &ControlBlock::fetch_add)
      .def("wait_any", &ControlBlock::wait_any)
      .def("wait_ge", &ControlBlock::wait_ge)
      .def("enqueue", &ControlBlock::enqueue, py::arg("stream"), py::arg("words"),
           py::arg("srcs") = std::vector<int64_t>{})
      .def("device_addr", &ControlBlock::device_addr)
      .def("enqueue_store", &ControlBlock::enqueue_store)
      .def("enqueue_store2", &ControlBlock::enqueue_store2)
      .def("enable_device_doorbells", &ControlBlock::enable_device_doorbells)
      .def_property_readonly("bell_mode", &ControlBlock::bell_mode)
      .def("wait_no_reader", &ControlBlock::wait_no_reader)
      .def("wait_no_reader_b", &ControlBlock::wait_no_reader_b)
      .def("heartbeat", &ControlBlock::heartbeat)
      .def("ps_beat", &ControlBlock::ps_beat)
      .def("ps_silent", &ControlBlock::ps_silent)
      .def_static("now_ns", &now_ns)
      .def_property_readonly("world", &ControlBlock::world)
      .def_property_readonly_static("SLOTS", [](py::object) { return kSlots; })
      .def_property_readonly_static("NPUB", [](py::object) { return kPub; })
      .def_property_readonly_static("MAX_BUCKETS", [](py::object) { return kMaxBuckets; });
  m.attr("F_PUSH_SEQ") = (int)PUSH_SEQ;
  m.attr("F_ACK_SEQ") = (int)ACK_SEQ;
  m.attr("F_PUSH_VER") = (int)PUSH_VER;
  m.attr("F_APPLIED_VER") = (int)APPLIED_VER;
  m.attr("F_STOP") = (int)STOP;
  m.attr("F_HEARTBEAT") = (int)HEARTBEAT;
  m.attr("F_INCL_SEQ") = (int)INCL_SEQ;
  m.attr("F_PUSH_FLAG") = (int)PUSH_FLAG;
  m.attr("F_READING") = (int)READING;
  m.attr("F_PULL_REQ") = (int)PULL_REQ;
  m.attr("F_SENT_VER") = (int)SENT_VER;
  m.attr("F_PUB_VER") = (int)PUB_VER;
  m.attr("F_PS_STOP") = (int)PS_STOP;
  m.attr("F_ERROR") = (int)ERROR;
  m.attr("F_DROPS") = (int)DROPS;
  m.attr("F_UPDATES") = (int)UPDATES;
  m.attr("F_BUF_VER") = (int)BUF_VER;
  m.attr("F_LAST_STALE") = (int)LAST_STALE;
  m.attr("F_LAST_STALE_SEQ") = (int)LAST_STALE_SEQ;
  m.attr("F_BPUB_VER") = (int)BPUB_VER;
  m.attr("F_BBUF_VER") = (int)BBUF_VER;
  m.attr("F_READING_B") = (int)READING_B;
  m.attr("F_OPEN_TURN") = (int)OPEN_TURN;
  m.attr("F_PS_HB") = (int)PS_HB;
  m.attr("F_PS_DEAD_NS") = (int)PS_DEAD_NS;
}

}  // namespace rt
}  // namespace hipps
