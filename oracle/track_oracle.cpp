// ORACLE — TEST INFRASTRUCTURE ONLY. CoarseTracker restatement (filled in below).
