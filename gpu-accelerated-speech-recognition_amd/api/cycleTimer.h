// Drop-in for the reference's cycleTimer.h (CycleTimer::currentSeconds(),
// used by main.cpp:13,78).  Monotonic std::chrono clock; one tick = 1 ns.
#ifndef ASR_API_CYCLE_TIMER_H_
#define ASR_API_CYCLE_TIMER_H_
#include <chrono>

class CycleTimer {
public:
    typedef unsigned long long SysClock;

    static SysClock currentTicks() {
        return (SysClock)std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch())
            .count();
    }
    static double currentSeconds() { return currentTicks() * secondsPerTick(); }
    static double ticksPerSecond() { return 1.0 / secondsPerTick(); }
    static const char* tickUnits() { return "ns"; }
    static double secondsPerTick() { return 1e-9; }
    static double msPerTick() { return secondsPerTick() * 1000.0; }

private:
    CycleTimer();
};
#endif
