// ORACLE — TEST INFRASTRUCTURE ONLY. ImmaturePoint::traceOn restatement (filled in below).
