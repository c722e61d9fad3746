// Signature stub of the rclcpp pieces the MinSnap adapter and the reference node use
// (tests/ros2_stub/README.md).  Declarations only: -fsyntax-only type checking.
#pragma once
#include <memory>
#include <string>
#include <vector>

namespace rclcpp {

class Time {
public:
    double seconds() const;
};

class Clock {
public:
    using SharedPtr = std::shared_ptr<Clock>;
    Time now();
};

class Logger {};
Logger get_logger(const std::string& name);

class Node {
public:
    template <class T>
    bool get_parameter(const std::string& name, T& value) const;
    template <class T>
    T declare_parameter(const std::string& name, const T& default_value);
    Clock::SharedPtr get_clock();
    Logger get_logger() const;
};

namespace detail {
void log(const Logger&, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
}

}  // namespace rclcpp

#define RCLCPP_INFO(logger, ...) ::rclcpp::detail::log((logger), __VA_ARGS__)
#define RCLCPP_WARN(logger, ...) ::rclcpp::detail::log((logger), __VA_ARGS__)
#define RCLCPP_ERROR(logger, ...) ::rclcpp::detail::log((logger), __VA_ARGS__)
