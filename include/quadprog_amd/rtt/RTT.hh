// RTT.hh — the slice of the Orocos RTT 2.x component surface the reference controller uses,
// so MotionGenerationQuadraticProgram can be deployed, connected and driven by port name the way
// the reference deployment script does (ops/mgqp.ops:180-236) without an Orocos installation
// (none exists in this image: SURVEY.md §8(c)).
//
// What the reference component touches (src/mgqp.cpp, include/mgqp.hpp:70-241):
//   * RTT::TaskContext with addOperation(name, &C::m, this, RTT::ClientThread).doc(...)
//     (src/mgqp.cpp:89-95), ports() -> addPort / removePort (:180-482), the hooks
//     configureHook/startHook/updateHook/stopHook/cleanupHook (mgqp.hpp:76-80);
//   * RTT::InputPort<T>::read(T&) -> RTT::FlowStatus {NoData, OldData, NewData}
//     (:874-916), InputPort/OutputPort::connected() (configureHook :142-170),
//     RTT::OutputPort<T>::write / setDataSample (:1165-1176, :413-470), RTT::ConnPolicy;
//   * ORO_CREATE_COMPONENT_LIBRARY() ORO_LIST_COMPONENT_TYPE(C) (:1270);
//   * from the deployer script: loadComponent, setActivity, operation calls by name and
//     connect("a.port", "b.port", cp) (ops/mgqp.ops:180-236).
// Semantics kept: a connection is a data object holding the last written sample (RTT's default
// ConnPolicy::DATA); read() returns NoData until the first write, NewData once per new sample,
// then OldData with the last sample copied out (copy_old_data = true, RTT's default); NoData
// leaves the caller's sample untouched.  An exception thrown by updateHook() puts the component
// in the Exception state (RTT's TaskCore behaviour), and update() on a component that is not
// Running does nothing.
#ifndef QUADPROG_AMD_RTT_HH
#define QUADPROG_AMD_RTT_HH

#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <typeinfo>
#include <utility>
#include <vector>

namespace RTT {

enum FlowStatus { NoData = 0, OldData = 1, NewData = 2 };
enum ExecutionThread { OwnThread, ClientThread };

struct ConnPolicy {  // only the default DATA connection type is modelled
  int type = 0;
  bool init = false;
};

class TaskContext;

namespace base {

class PortInterface {
 public:
  explicit PortInterface(std::string name) : name_(std::move(name)) {}
  virtual ~PortInterface() {}
  const std::string& getName() const { return name_; }
  PortInterface& doc(const std::string& d) {
    doc_ = d;
    return *this;
  }
  const std::string& getDescription() const { return doc_; }
  virtual bool connected() const = 0;
  virtual bool isInput() const = 0;
  virtual const std::type_info& type() const = 0;
  // connect this output port to `in` (both must carry the same type)
  virtual bool connectTo(PortInterface* in, const ConnPolicy& cp) = 0;
  virtual void disconnect() = 0;

 private:
  std::string name_, doc_;
};

}  // namespace base

namespace internal {
template <class T>
struct Channel {  // ConnPolicy::DATA: the last sample plus a "new" flag for the reader
  T sample{};
  bool written = false, fresh = false;
};
}  // namespace internal

template <class T>
class OutputPort;

template <class T>
class InputPort : public base::PortInterface {
 public:
  explicit InputPort(const std::string& name, const ConnPolicy& = ConnPolicy()) : PortInterface(name) {}
  ~InputPort() override { disconnect(); }

  FlowStatus read(T& sample, bool copy_old_data = true) {
    if (!ch_ || !ch_->written) return NoData;
    if (ch_->fresh) {
      ch_->fresh = false;
      sample = ch_->sample;
      return NewData;
    }
    if (copy_old_data) sample = ch_->sample;
    return OldData;
  }
  bool connected() const override { return static_cast<bool>(ch_); }
  bool isInput() const override { return true; }
  const std::type_info& type() const override { return typeid(T); }
  bool connectTo(base::PortInterface* other, const ConnPolicy& cp) override {
    return other && other->connectTo(this, cp);  // symmetric: let the output side wire it
  }
  void disconnect() override;

 private:
  friend class OutputPort<T>;
  std::shared_ptr<internal::Channel<T>> ch_;
  OutputPort<T>* writer_ = nullptr;
};

template <class T>
class OutputPort : public base::PortInterface {
 public:
  explicit OutputPort(const std::string& name, bool = true) : PortInterface(name) {}
  ~OutputPort() override { disconnect(); }

  void setDataSample(const T& sample) { sample_ = sample; }
  void write(const T& sample) {
    sample_ = sample;
    has_written_ = true;
    for (auto& c : chans_) {
      c->sample = sample;
      c->written = true;
      c->fresh = true;
    }
  }
  bool connected() const override { return !readers_.empty(); }
  bool isInput() const override { return false; }
  const std::type_info& type() const override { return typeid(T); }
  bool connectTo(base::PortInterface* other, const ConnPolicy& cp) override {
    auto* in = dynamic_cast<InputPort<T>*>(other);
    if (!in) return false;  // type mismatch or not an input port
    in->disconnect();       // an input port has one writer in this model
    auto ch = std::make_shared<internal::Channel<T>>();
    if (cp.init && has_written_) {  // ConnPolicy::init: hand over the last sample
      ch->sample = sample_;
      ch->written = ch->fresh = true;
    }
    in->ch_ = ch;
    in->writer_ = this;
    chans_.push_back(ch);
    readers_.push_back(in);
    return true;
  }
  bool connectTo(InputPort<T>& in, const ConnPolicy& cp = ConnPolicy()) { return connectTo(&in, cp); }
  void disconnect() override {
    for (auto* r : readers_) {
      r->ch_.reset();
      r->writer_ = nullptr;
    }
    readers_.clear();
    chans_.clear();
  }
  const T& lastSample() const { return sample_; }

 private:
  friend class InputPort<T>;
  void drop(InputPort<T>* in) {
    for (size_t i = 0; i < readers_.size(); ++i)
      if (readers_[i] == in) {
        readers_.erase(readers_.begin() + i);
        chans_.erase(chans_.begin() + i);
        return;
      }
  }
  T sample_{};
  bool has_written_ = false;
  std::vector<std::shared_ptr<internal::Channel<T>>> chans_;
  std::vector<InputPort<T>*> readers_;
};

template <class T>
void InputPort<T>::disconnect() {
  if (writer_) writer_->drop(this);
  writer_ = nullptr;
  ch_.reset();
}

// TaskContext::ports(): the component's named ports
class DataFlowInterface {
 public:
  // As RTT 2.x's DataFlowInterface::addLocalPort: a port added under a name that is already
  // present replaces it, and the replaced port is first removed, which disconnects it
  // (removeLocalPort -> PortInterface::disconnect()), even when it is the same port object.
  base::PortInterface& addPort(base::PortInterface& p) { return addPort(p.getName(), p); }
  base::PortInterface& addPort(const std::string& name, base::PortInterface& p) {
    removePort(name);
    ports_[name] = &p;
    return p;
  }
  bool removePort(const std::string& name) {
    auto it = ports_.find(name);
    if (it == ports_.end()) return false;
    it->second->disconnect();
    ports_.erase(it);
    return true;
  }
  base::PortInterface* getPort(const std::string& name) const {
    auto it = ports_.find(name);
    return it == ports_.end() ? nullptr : it->second;
  }
  std::vector<std::string> getPortNames() const {
    std::vector<std::string> v;
    for (const auto& kv : ports_) v.push_back(kv.first);
    return v;
  }

 private:
  std::map<std::string, base::PortInterface*> ports_;
};

// addOperation(...).doc(...): a named, type-checked callable
class OperationBase {
 public:
  virtual ~OperationBase() {}
  OperationBase& doc(const std::string& d) {
    doc_ = d;
    return *this;
  }
  const std::string& getDescription() const { return doc_; }
  ExecutionThread thread = ClientThread;

 private:
  std::string doc_;
};

template <class Sig>
class Operation : public OperationBase {
 public:
  explicit Operation(std::function<Sig> f) : fn(std::move(f)) {}
  std::function<Sig> fn;
};

class TaskContext {
 public:
  enum TaskState { Init, PreOperational, FatalError, Exception, Stopped, Running, RunTimeError };

  explicit TaskContext(const std::string& name) : name_(name) {}
  virtual ~TaskContext() {}

  const std::string& getName() const { return name_; }
  DataFlowInterface* ports() { return &ports_; }
  const DataFlowInterface* ports() const { return &ports_; }
  TaskState getTaskState() const { return state_; }
  bool isRunning() const { return state_ == Running; }
  const std::string& lastException() const { return last_exception_; }

  template <class C, class R, class... A>
  OperationBase& addOperation(const std::string& name, R (C::*m)(A...), C* obj,
                              ExecutionThread et = ClientThread) {
    auto op = std::make_shared<Operation<R(A...)>>(
        [obj, m](A... a) -> R { return (obj->*m)(std::forward<A>(a)...); });
    op->thread = et;
    ops_[name] = op;
    return *op;
  }
  // a registered operation, by name and signature (std::bad_cast-free: nullptr on mismatch)
  template <class Sig>
  std::function<Sig> getOperation(const std::string& name) const {
    auto it = ops_.find(name);
    if (it == ops_.end()) throw std::out_of_range("no operation '" + name + "' in " + name_);
    auto* op = dynamic_cast<Operation<Sig>*>(it->second.get());
    if (!op) throw std::invalid_argument("operation '" + name + "' called with the wrong signature");
    return op->fn;
  }
  std::vector<std::string> getOperationNames() const {
    std::vector<std::string> v;
    for (const auto& kv : ops_) v.push_back(kv.first);
    return v;
  }

  // TaskCore state machine
  bool configure() {
    if (state_ != PreOperational && state_ != Stopped && state_ != Init) return false;
    const bool ok = configureHook();
    state_ = ok ? Stopped : PreOperational;
    return ok;
  }
  bool start() {
    if (state_ != Stopped) return false;
    if (!startHook()) return false;
    state_ = Running;
    return true;
  }
  // one activity trigger (the periodic activity's step, ops/mgqp.ops:182)
  bool update() {
    if (state_ != Running) return false;
    try {
      updateHook();
    } catch (const std::exception& e) {
      last_exception_ = e.what();
      state_ = Exception;
      exceptionHook();
      return false;
    }
    return true;
  }
  bool stop() {
    if (state_ != Running) return false;
    stopHook();
    state_ = Stopped;
    return true;
  }
  bool cleanup() {
    if (state_ != Stopped) return false;
    cleanupHook();
    state_ = PreOperational;
    return true;
  }
  bool recover() {
    if (state_ != Exception) return false;
    state_ = Stopped;
    return true;
  }
  void setPeriod(double seconds) { period_ = seconds; }
  double getPeriod() const { return period_; }

 protected:
  virtual bool configureHook() { return true; }
  virtual bool startHook() { return true; }
  virtual void updateHook() {}
  virtual void stopHook() {}
  virtual void cleanupHook() {}
  virtual void exceptionHook() {}

 private:
  std::string name_;
  DataFlowInterface ports_;
  std::map<std::string, std::shared_ptr<OperationBase>> ops_;
  TaskState state_ = PreOperational;
  std::string last_exception_;
  double period_ = 0.0;
};

// ---- component factory (ORO_CREATE_COMPONENT_LIBRARY / ORO_LIST_COMPONENT_TYPE) -------------
namespace ComponentFactories {
using Factory = TaskContext* (*)(const std::string& name);
inline std::map<std::string, Factory>& Instance() {
  static std::map<std::string, Factory> f;
  return f;
}
}  // namespace ComponentFactories

template <class C>
struct ComponentFactoryRegistration {
  explicit ComponentFactoryRegistration(const char* type) {
    ComponentFactories::Instance()[type] = [](const std::string& name) -> TaskContext* {
      return new C(name);
    };
  }
};

// The deployer's script commands (ops/mgqp.ops): loadComponent, setActivity, connect
class Deployer {
 public:
  bool loadComponent(const std::string& name, const std::string& type) {
    auto& f = ComponentFactories::Instance();
    auto it = f.find(type);
    if (it == f.end() || comps_.count(name)) return false;
    comps_[name].reset(it->second(name));
    return true;
  }
  // a component created elsewhere (peers of the deployment: sources, sinks)
  void addPeer(TaskContext* tc) { peers_[tc->getName()] = tc; }
  TaskContext* getPeer(const std::string& name) const {
    auto it = comps_.find(name);
    if (it != comps_.end()) return it->second.get();
    auto jt = peers_.find(name);
    return jt == peers_.end() ? nullptr : jt->second;
  }
  bool setActivity(const std::string& name, double period, int /*priority*/ = 0, int /*sched*/ = 0) {
    TaskContext* tc = getPeer(name);
    if (!tc) return false;
    tc->setPeriod(period);
    return true;
  }
  // connect("component.port", "component.port", cp): output -> input, in either order
  bool connect(const std::string& a, const std::string& b, const ConnPolicy& cp = ConnPolicy()) {
    base::PortInterface* pa = port(a);
    base::PortInterface* pb = port(b);
    if (!pa || !pb || pa->isInput() == pb->isInput()) return false;
    base::PortInterface* out = pa->isInput() ? pb : pa;
    base::PortInterface* in = pa->isInput() ? pa : pb;
    return out->connectTo(in, cp);
  }

 private:
  base::PortInterface* port(const std::string& qualified) const {
    const size_t dot = qualified.find('.');
    if (dot == std::string::npos) return nullptr;
    TaskContext* tc = getPeer(qualified.substr(0, dot));
    return tc ? tc->ports()->getPort(qualified.substr(dot + 1)) : nullptr;
  }
  std::map<std::string, std::unique_ptr<TaskContext>> comps_;
  std::map<std::string, TaskContext*> peers_;
};

}  // namespace RTT

#define ORO_CREATE_COMPONENT_LIBRARY()
#define ORO_LIST_COMPONENT_TYPE(C) \
  static ::RTT::ComponentFactoryRegistration<C> oro_component_registration_##C(#C);

#endif
